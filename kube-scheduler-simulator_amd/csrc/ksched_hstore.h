// Stores into a pinned, fine-grained host block (the per-cycle kernel and the
// topology kernel's per-cycle capture write their rows straight into it).
// Included by ksched_dev.h inside namespace ksk.
#pragma once

// Stores into the host block.  SYS: system-scope relaxed stores (global_store
// sc0 sc1: written through to the fine-grained host memory, nothing left in
// L2), so a vmcnt(0) wait orders them before the flag and no L2 write-back
// (buffer_wbl2) is needed; else plain stores + __threadfence_system.
template <bool SYS, class T>
__device__ __forceinline__ void hst(T* p, T v) {
  if constexpr (SYS) __hip_atomic_store((__attribute__((address_space(1))) T*)p, v, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_SYSTEM);
  else *p = v;
}
template <bool SYS>
__device__ __forceinline__ void cyc_put(char* base, size_t idx, int64_t v, bool narrow) {
  if (narrow) hst<SYS>(reinterpret_cast<int32_t*>(base) + idx, (int32_t)v);
  else hst<SYS>(reinterpret_cast<int64_t*>(base) + idx, v);
}
template <bool SYS>
__device__ __forceinline__ void cyc_put_es(char* base, size_t idx, int64_t v, int es) {
  if (es == 1) hst<SYS>(reinterpret_cast<uint8_t*>(base) + idx, (uint8_t)v);
  else if (es == 2) hst<SYS>(reinterpret_cast<int16_t*>(base) + idx, (int16_t)v);
  else cyc_put<SYS>(base, idx, v, es == 4);
}

// Every host store of this wave performed before what follows (the arrival,
// the flag).
template <bool SYS>
__device__ __forceinline__ void host_release() {
  if constexpr (SYS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else __threadfence_system();
}

