// Checks the lane exchanges behind bq_device.h's line-covering stores on the
// GPU: lane L holds K consecutive candles (K = 4: two 16-byte pieces, K = 8:
// four); after the exchange, register m of lane L must hold the piece whose
// candle offset store_offset<K>(L) + 128 m it is stored at, so that each
// store instruction covers candles [128 m, 128 m + 128) of the wave's slice.
// Build: hipcc -O3 --offload-arch=gfx950 -Ibinquant_amd/csrc -Iinclude tools/permlane_check.hip -o tools/permlane_check
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "bq_device.h"

template <int K>
__global__ void check(int* bad) {
  const int lane = threadIdx.x;
  double x[K];
  for (int k = 0; k < K; ++k) x[k] = (double)(K * lane + k);
  bq::dbl2 p[K / 2];
  for (int j = 0; j < K / 2; ++j) p[j] = bq::dbl2{x[2 * j], x[2 * j + 1]};
  bq::line_exchange<K>(p);
  const int o = bq::line_offset<K>(lane);
  for (int m = 0; m < K / 2; ++m) {
    const double want = (double)(128 * m + o);
    if (p[m].x != want || p[m].y != want + 1.0) atomicAdd(bad, 1);
  }
}

int main() {
  int* bad;
  hipMalloc(&bad, sizeof(int));
  int h = 0;
  hipMemset(bad, 0, sizeof(int));
  check<4><<<1, 64>>>(bad);
  hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost);
  printf("K=4 mismatches: %d\n", h);
  int fails = h;
  hipMemset(bad, 0, sizeof(int));
  check<8><<<1, 64>>>(bad);
  hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost);
  printf("K=8 mismatches: %d\n", h);
  fails += h;
  printf(fails ? "PERMLANE_CHECK_FAILED\n" : "PERMLANE_CHECK_OK\n");
  return fails ? 1 : 0;
}
