// The kernel instantiations compiled outside the host TU, one group per part
// (ksched_part.hip -DKSG_PART=k): explicit instantiation definitions there,
// explicit instantiation declarations in ksched.hip, so the host TU launches
// them by their stubs and never compiles them.  A launch of an instantiation
// missing here is compiled in the host TU as before.
#pragma once

#ifdef KSG_PART
#define KSG_INST template __global__ void
#else
#define KSG_INST extern template __global__ void
#endif

namespace ksk {

#if !defined(KSG_PART) || KSG_PART == 1
KSG_INST ksg_topo_coop<1, false, 0>(CoopArgs);
KSG_INST ksg_topo_coop<1, false, 1>(CoopArgs);
KSG_INST ksg_topo_coop<1, false, 2>(CoopArgs);
KSG_INST ksg_topo_coop<1, true, 0>(CoopArgs);
KSG_INST ksg_topo_coop<1, true, 1>(CoopArgs);
KSG_INST ksg_topo_coop<1, true, 2>(CoopArgs);
#endif
#if !defined(KSG_PART) || KSG_PART == 4
KSG_INST ksg_topo_coop<1, false, 3>(CoopArgs);
KSG_INST ksg_topo_coop<1, true, 3>(CoopArgs);
#endif
#if !defined(KSG_PART) || KSG_PART == 2
KSG_INST ksg_topo_coop<2, false, 0>(CoopArgs);
KSG_INST ksg_topo_coop<2, false, 1>(CoopArgs);
KSG_INST ksg_topo_coop<2, false, 2>(CoopArgs);
KSG_INST ksg_topo_coop<4, false, 0>(CoopArgs);
#endif
#if !defined(KSG_PART) || KSG_PART == 3
KSG_INST ksg_topo_coop<4, false, 1>(CoopArgs);
KSG_INST ksg_topo_coop<4, false, 2>(CoopArgs);
KSG_INST ksg_topo_coop<8, false, 0>(CoopArgs);
#endif
#if !defined(KSG_PART) || KSG_PART == 4
KSG_INST ksg_topo_coop<16, false, 0>(CoopArgs);
KSG_INST ksg_topo_coop<32, false, 0>(CoopArgs);
#endif
#if !defined(KSG_PART) || KSG_PART == 5
KSG_INST ksg_sweep<256, 0, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 0, false, true, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 0, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 0, true, false, false, true>(SweepArgs);
KSG_INST ksg_sweep<256, 0, true, false, true, false>(SweepArgs);
KSG_INST ksg_sweep<256, 0, true, false, true, true>(SweepArgs);
KSG_INST ksg_sweep<256, 0, true, true, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 0, true, true, false, true>(SweepArgs);
KSG_INST ksg_sweep<256, 0, true, true, true, false>(SweepArgs);
KSG_INST ksg_sweep<256, 0, true, true, true, true>(SweepArgs);
KSG_INST ksg_sweep<1024, 0, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<1024, 0, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<1024, 0, true, false, false, true>(SweepArgs);
KSG_INST ksg_sweep<1024, 0, true, false, true, false>(SweepArgs);
KSG_INST ksg_sweep<1024, 0, true, false, true, true>(SweepArgs);
KSG_INST ksg_sweep<256, 8, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 8, false, true, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 8, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 8, true, false, false, true>(SweepArgs);
KSG_INST ksg_sweep<256, 8, true, false, true, false>(SweepArgs);
KSG_INST ksg_sweep<256, 8, true, false, true, true>(SweepArgs);
KSG_INST ksg_sweep<256, 8, true, true, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 8, true, true, false, true>(SweepArgs);
KSG_INST ksg_sweep<256, 8, true, true, true, false>(SweepArgs);
KSG_INST ksg_sweep<256, 8, true, true, true, true>(SweepArgs);
#endif
#if !defined(KSG_PART) || KSG_PART == 6
KSG_INST ksg_sweep<256, 16, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 16, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 16, true, false, false, true>(SweepArgs);
KSG_INST ksg_sweep<256, 20, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 20, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 20, true, false, false, true>(SweepArgs);
KSG_INST ksg_sweep<256, 24, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 24, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 24, true, false, false, true>(SweepArgs);
#endif
#if !defined(KSG_PART) || KSG_PART == 7
KSG_INST ksg_sweep<256, 32, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 32, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<256, 32, true, false, false, true>(SweepArgs);
KSG_INST ksg_sweep<512, 32, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<512, 32, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<512, 32, true, false, false, true>(SweepArgs);
KSG_INST ksg_sweep<1024, 32, false, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<1024, 32, true, false, false, false>(SweepArgs);
KSG_INST ksg_sweep<1024, 32, true, false, false, true>(SweepArgs);
#endif

}  // namespace ksk

#undef KSG_INST
