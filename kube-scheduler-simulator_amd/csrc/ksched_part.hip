// One part of libksched.so's device code (__graft_entry__.build compiles this
// file once per -DKSG_PART=k, in parallel with the host TU ksched.hip): the
// explicit instantiations ksched_parts.h lists for part k.
#if !defined(KSG_PART)
#error "compile with -DKSG_PART=<1..7>"
#endif
#if KSG_PART <= 4
#define KSG_WITH_TOPO 1   // ksg_topo_coop (which uses the sweep's helpers)
#endif
#define KSG_WITH_SWEEP 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "ksched_dev.h"
#include "ksched_parts.h"
