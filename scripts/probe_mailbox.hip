// Measurement probe (not product): round trip of a host -> GPU call and the
// GPU -> host completion word, with the call's mailbox in (A) pinned host
// memory (the per-cycle server's current form) or (B) fine-grained device
// memory the CPU writes through the BAR.  One persistent workgroup of 64
// lanes polls the mailbox's sequence word, reads a 640-byte call with all
// lanes, and stores the sequence number into a pinned host completion word.
// The kernel leaves on a stop word or after a bounded number of polls.
//
//   hipcc --offload-arch=gfx950 -O2 -o probe_mailbox scripts/probe_mailbox.hip
//   ./probe_mailbox [iters]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

struct Box {
  unsigned seq;
  unsigned stop;
  unsigned pad[30];
  int call[160];   // 640 bytes
};

template <class T>
__device__ __forceinline__ T sys_ld(const T* p) {
  return __hip_atomic_load((T*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void server(const Box* box, unsigned* done, int* sink, int read_call) {
  __shared__ int s_call[160];
  unsigned last = 0;
  const int lane = threadIdx.x;
  for (;;) {
    unsigned seq = last;
    unsigned long long spins = 0;
    if (lane == 0) {
      for (;;) {
        seq = sys_ld(&box->seq);
        if (seq != last || sys_ld(&box->stop)) break;
        if (++spins > (1ull << 26)) break;   // bounded: the kernel always ends
        __builtin_amdgcn_s_sleep(1);
      }
    }
    seq = (unsigned)__builtin_amdgcn_readfirstlane((int)seq);
    if (seq == last) break;
    if (read_call) {
      int a = sys_ld(&box->call[lane]), b = sys_ld(&box->call[lane + 64]), c = lane < 32 ? sys_ld(&box->call[lane + 128]) : 0;
      s_call[lane] = a;
      s_call[lane + 64] = b;
      if (lane < 32) s_call[lane + 128] = c;
      __syncthreads();
      if (lane == 0) sink[0] = s_call[7] + s_call[150];
    }
    if (lane == 0) __hip_atomic_store(done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    last = seq;
  }
}

static double run(Box* hbox, const Box* dbox, unsigned* hdone, unsigned* ddone, int* sink, int iters, int read_call,
                  hipStream_t st) {
  std::memset((void*)hbox, 0, 128);
  *(volatile unsigned*)hdone = 0;
  hipLaunchKernelGGL(server, dim3(1), dim3(64), 0, st, dbox, ddone, sink, read_call);
  CK(hipGetLastError());
  double total = 0;
  for (int i = 1; i <= iters; i++) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < 160; k++) hbox->call[k] = i + k;
    __builtin_ia32_sfence();
    __atomic_store_n(&hbox->seq, (unsigned)i, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
    while (__atomic_load_n((volatile unsigned*)hdone, __ATOMIC_ACQUIRE) != (unsigned)i) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {   // the kernel left: stop
        std::printf("no completion for call %d\n", i);
        __atomic_store_n(&hbox->stop, 1u, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(st));
        return -1;
      }
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (i > 100) total += std::chrono::duration<double, std::micro>(t1 - t0).count();
  }
  __atomic_store_n(&hbox->stop, 1u, __ATOMIC_RELEASE);
  __builtin_ia32_sfence();
  CK(hipStreamSynchronize(st));
  return total / (iters - 100);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 5000;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  unsigned* hdone;
  CK(hipHostMalloc((void**)&hdone, 64, hipHostMallocMapped | hipHostMallocCoherent));
  unsigned* ddone;
  CK(hipHostGetDevicePointer((void**)&ddone, hdone, 0));
  int* sink;
  CK(hipMalloc((void**)&sink, 64));
  // (A) pinned host mailbox
  Box* hA;
  CK(hipHostMalloc((void**)&hA, sizeof(Box), hipHostMallocMapped | hipHostMallocCoherent));
  Box* dA;
  CK(hipHostGetDevicePointer((void**)&dA, hA, 0));
  for (int rc = 0; rc < 2; rc++)
    std::printf("host-pinned mailbox, read_call=%d: %.2f us per round trip\n", rc, run(hA, dA, hdone, ddone, sink, iters, rc, st));
  // (B) fine-grained device memory written by the CPU
  Box* dB = nullptr;
  hipError_t e = hipExtMallocWithFlags((void**)&dB, sizeof(Box), hipDeviceMallocFinegrained);
  if (e != hipSuccess) {
    std::printf("fine-grained device malloc: %s\n", hipGetErrorString(e));
    return 0;
  }
  hipPointerAttribute_t attr;
  CK(hipPointerGetAttributes(&attr, dB));
  std::printf("fine-grained device buffer: type %d, device %d, host pointer %p, device pointer %p\n",
              (int)attr.type, attr.device, attr.hostPointer, attr.devicePointer);
  Box* hB = attr.hostPointer ? (Box*)attr.hostPointer : dB;   // (large BAR: the same address on the CPU)
  std::fflush(stdout);
  // a CPU write and read-back before any kernel runs (a fault here ends the
  // process with nothing on the GPU)
  ((volatile unsigned*)hB)[2] = 0x5a5a5a5au;
  std::printf("CPU write/read of the device buffer: %s\n", ((volatile unsigned*)hB)[2] == 0x5a5a5a5au ? "ok" : "MISMATCH");
  for (int rc = 0; rc < 2; rc++)
    std::printf("device fine-grained mailbox, read_call=%d: %.2f us per round trip\n", rc,
                run(hB, dB, hdone, ddone, sink, iters, rc, st));
  return 0;
}
