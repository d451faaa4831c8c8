// Accuracy of the hardware fp64 reciprocal on gfx950, alone and after one /
// two Newton steps, against the IEEE quotient 1 / x, over x = m * 2^e with
// random mantissas and e in [-60, 60]: max relative error of each form.
// (bq_context.hip's cx_div: how many Newton steps the 1e-9 contract needs.)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>

__global__ void probe(const double* x, double* e0, double* e1, double* e2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i], q = 1.0 / v;
  double r = __builtin_amdgcn_rcp(v);
  e0[i] = fabs(r - q) / q;
  r = fma(r, fma(-v, r, 1.0), r);
  e1[i] = fabs(r - q) / q;
  r = fma(r, fma(-v, r, 1.0), r);
  e2[i] = fabs(r - q) / q;
}

int main() {
  const int n = 1 << 22;
  double* h = (double*)malloc(n * sizeof(double));
  srand(7);
  for (int i = 0; i < n; ++i) {
    const double m = 1.0 + (double)rand() / RAND_MAX + (double)rand() / RAND_MAX / 4294967296.0;
    h[i] = ldexp(m, (rand() % 121) - 60);
  }
  double *x, *e[3];
  hipMalloc(&x, n * sizeof(double));
  for (int k = 0; k < 3; ++k) hipMalloc(&e[k], n * sizeof(double));
  hipMemcpy(x, h, n * sizeof(double), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(n / 256), dim3(256), 0, 0, x, e[0], e[1], e[2], n);
  for (int k = 0; k < 3; ++k) {
    hipMemcpy(h, e[k], n * sizeof(double), hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < n; ++i) mx = h[i] > mx ? h[i] : mx;
    printf("newton steps %d: max relative error %.3e (2^%.1f)\n", k, mx, mx > 0 ? log2(mx) : -1e9);
  }
  return 0;
}
