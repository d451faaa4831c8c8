// Time-parallel ("panel mode") rolling sums / means and ewm for
// bq_rolling_batch (bq_panel.hip). Internal to the library: the C ABI entry is
// bq_rolling_batch with bq_roll_job.panel = 1.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace bq {

struct PanelJob {
  const double* x;
  double* out;
  int64_t ld_in, ld_out, rows;
  int win, minp, shift, mode;   // mode: BQ_ROLL_SUM / BQ_ROLL_MEAN / BQ_ROLL_EWM
  double alpha;
  const double *hi, *lo;        // ewm only: non-null = the series is the true range of
                                // (hi, lo, x = close), [S][ld_in] like x
};

constexpr int PN_MAXJOBS = 16;

struct PanelBatch {
  PanelJob j[PN_MAXJOBS];
  int64_t S;
  int T;
};

// launches the window jobs and the ewm jobs of a batch (n <= PN_MAXJOBS)
void launch_panel(const PanelBatch& B, int n, hipStream_t st);

// a job the panel kernels take: sum / mean with window + shift <= 128, ewm
bool panel_supported(int mode, int window, int shift);

}  // namespace bq
