// Accuracy probe of the device exp / log the log-space recursions use
// (lt_kernels.h lt_exp, lt_log, lt_log_acc) against the host's double
// functions: max and mean (bias) error in ulps of the result. Diagnostic.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../last_torch_amd/csrc/lt_kernels.h"

__global__ void probe(const float* x, float* e, float* l, float* la, float* lp, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  e[i] = lt_exp(x[i]);
  const float y = -x[i];  // log of values in (0, ...]: use exp of x as the argument
  (void)y;
  const float a = 1.f + __expf(x[i]) * 0.f + (float)(i % 97) / 3.f;  // [1, 33]
  l[i] = lt_log(a);
  la[i] = lt_log_acc(a);
  lp[i] = a;
}

int main() {
  const int n = 1 << 20;
  std::vector<float> x(n), e(n), l(n), la(n), lp(n);
  for (int i = 0; i < n; ++i) x[i] = -8.f * (float)i / n;  // exp arguments in (-8, 0]
  float *dx, *de, *dl, *dla, *dlp;
  hipMalloc(&dx, 4 * n); hipMalloc(&de, 4 * n); hipMalloc(&dl, 4 * n); hipMalloc(&dla, 4 * n);
  hipMalloc(&dlp, 4 * n);
  hipMemcpy(dx, x.data(), 4 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, dx, de, dl, dla, dlp, n);
  hipMemcpy(e.data(), de, 4 * n, hipMemcpyDeviceToHost);
  hipMemcpy(l.data(), dl, 4 * n, hipMemcpyDeviceToHost);
  hipMemcpy(la.data(), dla, 4 * n, hipMemcpyDeviceToHost);
  hipMemcpy(lp.data(), dlp, 4 * n, hipMemcpyDeviceToHost);
  double emax = 0, esum = 0, lmax = 0, lsum = 0, amax = 0, asum = 0;
  for (int i = 0; i < n; ++i) {
    const double re = std::exp((double)x[i]);
    const double d = ((double)e[i] - re) / re;  // relative
    emax = std::fmax(emax, std::fabs(d)); esum += d;
    const double rl = std::log((double)lp[i]);
    const double dl2 = (double)l[i] - rl, da = (double)la[i] - rl;
    lmax = std::fmax(lmax, std::fabs(dl2)); lsum += dl2;
    amax = std::fmax(amax, std::fabs(da)); asum += da;
  }
  std::printf("lt_exp on (-8, 0]: max rel err %.3e, mean rel err (bias) %.3e\n", emax, esum / n);
  std::printf("lt_log on [1, 33]: max abs err %.3e, mean abs err (bias) %.3e\n", lmax, lsum / n);
  std::printf("lt_log_acc on [1, 33]: max abs err %.3e, mean abs err (bias) %.3e\n", amax, asum / n);
  return 0;
}
