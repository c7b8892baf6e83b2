// clock_probe.hip -- the shader clock of a CU, measured (dev tool; built by
// `make probe` into build/libclock_probe.so, never loaded by the product).
// One wave spins until `ticks` shader-clock ticks (s_memtime) have passed and
// records the 100 MHz constant clock (s_memrealtime) across the same window:
// f = d(memtime) / d(memrealtime) x 100 MHz. tools/clock_probe.py launches it
// between lattice calls to show the clock the calls ran at, and the latency
// of uncached loads (a dependent chain) at the same moment.
#include <hip/hip_runtime.h>

__global__ void clock_probe_kernel(long long* out, long long ticks, const int* chain) {
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  const long long r0 = (long long)__builtin_amdgcn_s_memrealtime();
  long long t1 = t0;
  while (t1 - t0 < ticks) t1 = (long long)__builtin_amdgcn_s_memtime();
  const long long r1 = (long long)__builtin_amdgcn_s_memrealtime();
  // then 256 dependent loads through `chain` that bypass the caches (sc0
  // sc1): the memory round-trip latency, in 100 MHz ticks for all of them
  int idx = 0;
  const long long r2 = (long long)__builtin_amdgcn_s_memrealtime();
  for (int k = 0; k < 256; ++k) {
    int v;
    const int* p = chain + idx;
    asm volatile("global_load_dword %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    idx = v;
  }
  const long long r3 = (long long)__builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = r1 - r0;
    out[2] = r3 - r2 + (idx & 0);  // idx keeps the chain live
    out[3] = idx;
  }
}

extern "C" int clock_probe(long long* out, long long ticks, const int* chain, void* stream) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out, ticks,
                     chain);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
