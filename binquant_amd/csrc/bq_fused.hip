// Fused element-wise programs (bq_fused_eval, include/binquant_amd.h): the
// element-wise glue between the rolling series of the strategy pipelines
//  as one launch per stage instead of one torch kernel
// per operator, each of which reads and writes a whole [S, T] fp64 panel.
//
// Mapping: 256 threads = 256 consecutive candles of one symbol (coalesced
// loads / stores, shifted loads are offset rows of the same lines). The
// program is wave-uniform: instructions and operand descriptors are read
// from the kernarg segment with scalar loads and dispatched by a scalar
// branch. Program registers live in LDS ([reg][thread], conflict-free);
// the loads are issued together first (up to 16 in flight per thread) so a
// thread waits for HBM once, not once per operand. Arithmetic is plain IEEE
// fp64 (-ffp-contract=off: no FMA contraction), in the program's order.
// Constant operands are read from the kernarg table directly (no register).
#include "bq_device.h"
#include "binquant_amd.h"

namespace bq {

constexpr int FU_NT = 256;

__device__ __forceinline__ double fused_load(const bq_fused_operand& X, int64_t sym, int ts) {
  const int64_t off = sym * X.stride_s + (int64_t)ts * X.stride_t;
  return X.dtype == BQ_F_U8 ? (double)(static_cast<const uint8_t*>(X.ptr)[off] != 0)
                            : static_cast<const double*>(X.ptr)[off];
}

__global__ __launch_bounds__(FU_NT) void fused_kernel(const bq_fused_program P, int T, int nbt) {
  __shared__ double R[BQ_FUSED_MAX_REGS * FU_NT];
  const int tid = threadIdx.x;
  const int64_t sym = blockIdx.x / nbt;
  const int t = (int)(blockIdx.x % nbt) * FU_NT + tid;
  const bool live = t < T;
  auto reg = [&](uint64_t r) -> double& { return R[(int)r * FU_NT + tid]; };

  // loads first, all in flight together
  double lv[BQ_FUSED_MAX_LOADS];
#pragma unroll
  for (int i = 0; i < BQ_FUSED_MAX_LOADS; ++i) {
    if (i < P.n_loads) {
      const uint64_t in = P.ins[i];
      const int b = (int)((in >> 24) & 0xff), c = (int)((in >> 32) & 0xff);
      const int ts = t - (int)((int64_t)in >> 40);
      lv[i] = (live && ts >= 0 && ts < T) ? fused_load(P.in[b], sym, ts) : P.consts[c];
    }
  }
#pragma unroll
  for (int i = 0; i < BQ_FUSED_MAX_LOADS; ++i)
    if (i < P.n_loads) reg((P.ins[i] >> 8) & 0xff) = lv[i];

  for (int pc = P.n_loads; pc < P.n_ins; ++pc) {
    const uint64_t in = P.ins[pc];
    const int op = (int)(in & 0xff);
    const uint64_t d = (in >> 8) & 0xff, a = (in >> 16) & 0xff, b = (in >> 24) & 0xff, c = (in >> 32) & 0xff;
    const int imm = (int)((int64_t)in >> 40);
    // operands of the arithmetic ops: a register, or a constant (flag bits 40-42)
    auto opd = [&](uint64_t r, int k) -> double { return ((in >> (40 + k)) & 1) ? P.consts[r] : reg(r); };
    double r = 0.0;
    switch (op) {
      case BQ_F_LD: {   // a load after the first block (programs with > 16 loads)
        const int ts = t - imm;
        r = (live && ts >= 0 && ts < T) ? fused_load(P.in[b], sym, ts) : P.consts[c];
        break;
      }
      case BQ_F_CONST: r = P.consts[imm]; break;
      case BQ_F_INRANGE: r = (t - imm >= 0 && t - imm < T) ? 1.0 : 0.0; break;
      case BQ_F_ADD: r = opd(a, 0) + opd(b, 1); break;
      case BQ_F_SUB: r = opd(a, 0) - opd(b, 1); break;
      case BQ_F_MUL: r = opd(a, 0) * opd(b, 1); break;
      case BQ_F_DIV: r = opd(a, 0) / opd(b, 1); break;
      case BQ_F_FMAX: r = fmax(opd(a, 0), opd(b, 1)); break;
      case BQ_F_FMIN: r = fmin(opd(a, 0), opd(b, 1)); break;
      case BQ_F_MAXIMUM: {
        const double x = opd(a, 0), y = opd(b, 1);
        r = (x != x || y != y) ? qnan() : (x > y ? x : y);
        break;
      }
      case BQ_F_MINIMUM: {
        const double x = opd(a, 0), y = opd(b, 1);
        r = (x != x || y != y) ? qnan() : (x < y ? x : y);
        break;
      }
      case BQ_F_GT: r = opd(a, 0) > opd(b, 1) ? 1.0 : 0.0; break;
      case BQ_F_GE: r = opd(a, 0) >= opd(b, 1) ? 1.0 : 0.0; break;
      case BQ_F_LT: r = opd(a, 0) < opd(b, 1) ? 1.0 : 0.0; break;
      case BQ_F_LE: r = opd(a, 0) <= opd(b, 1) ? 1.0 : 0.0; break;
      case BQ_F_EQ: r = opd(a, 0) == opd(b, 1) ? 1.0 : 0.0; break;
      case BQ_F_NE: r = opd(a, 0) != opd(b, 1) ? 1.0 : 0.0; break;
      case BQ_F_AND: r = (opd(a, 0) != 0.0 && opd(b, 1) != 0.0) ? 1.0 : 0.0; break;
      case BQ_F_OR: r = (opd(a, 0) != 0.0 || opd(b, 1) != 0.0) ? 1.0 : 0.0; break;
      case BQ_F_NOT: r = opd(a, 0) != 0.0 ? 0.0 : 1.0; break;
      case BQ_F_ABS: r = fabs(opd(a, 0)); break;
      case BQ_F_NEG: r = -opd(a, 0); break;
      case BQ_F_ISNAN: {
        const double x = opd(a, 0);
        r = x != x ? 1.0 : 0.0;
        break;
      }
      case BQ_F_SQRT: r = sqrt(opd(a, 0)); break;
      case BQ_F_LOG: r = log(opd(a, 0)); break;
      case BQ_F_WHERE: r = opd(a, 0) != 0.0 ? opd(b, 1) : opd(c, 2); break;
      case BQ_F_ST: {
        if (live) {
          const bq_fused_operand& Y = P.out[imm];
          const int64_t off = sym * Y.stride_s + (int64_t)t * Y.stride_t;
          const double x = reg(a);
          if (Y.dtype == BQ_F_U8) static_cast<uint8_t*>(const_cast<void*>(Y.ptr))[off] = x != 0.0;
          else static_cast<double*>(const_cast<void*>(Y.ptr))[off] = x;
        }
        continue;
      }
      default: break;
    }
    reg(d) = r;
  }
}

}  // namespace bq

namespace {

int arity(int op) {
  switch (op) {
    case BQ_F_LD: case BQ_F_CONST: case BQ_F_INRANGE: return 0;
    case BQ_F_NOT: case BQ_F_ABS: case BQ_F_NEG: case BQ_F_ISNAN: case BQ_F_SQRT: case BQ_F_LOG: case BQ_F_ST:
      return 1;
    case BQ_F_WHERE: return 3;
    default: return 2;
  }
}

bool operand_ok(const bq_fused_operand& X) {
  return X.ptr && (X.dtype == BQ_F_F64 || X.dtype == BQ_F_U8) && X.stride_s >= 0 && X.stride_t >= 0;
}

}  // namespace

extern "C" {

int bq_fused_eval(const bq_fused_program* P, int64_t S, int64_t T, void* stream) {
  using namespace bq;
  if (!P || S < 0 || T < 0 || T > 0x7fffffff) return BQ_EINVAL;
  if (P->n_ins < 0 || P->n_ins > BQ_FUSED_MAX_INS || P->n_loads < 0 || P->n_loads > BQ_FUSED_MAX_LOADS ||
      P->n_loads > P->n_ins || P->n_regs < 0 || P->n_regs > BQ_FUSED_MAX_REGS || P->n_in < 0 ||
      P->n_in > BQ_FUSED_MAX_IN || P->n_out < 0 || P->n_out > BQ_FUSED_MAX_OUT || P->n_const < 0 ||
      P->n_const > BQ_FUSED_MAX_CONST)
    return BQ_EINVAL;
  for (int i = 0; i < P->n_in; ++i)
    if (!operand_ok(P->in[i])) return BQ_EINVAL;
  for (int i = 0; i < P->n_out; ++i)
    if (!operand_ok(P->out[i])) return BQ_EINVAL;
  for (int pc = 0; pc < P->n_ins; ++pc) {
    const uint64_t in = P->ins[pc];
    const int op = (int)(in & 0xff);
    const int d = (int)((in >> 8) & 0xff), a = (int)((in >> 16) & 0xff), b = (int)((in >> 24) & 0xff),
              c = (int)((in >> 32) & 0xff);
    const int64_t imm = (int64_t)in >> 40;
    if (op < BQ_F_LD || op > BQ_F_ST) return BQ_EINVAL;
    if (pc < P->n_loads && op != BQ_F_LD) return BQ_EINVAL;   // the load block comes first
    if (op != BQ_F_ST && d >= P->n_regs) return BQ_EINVAL;
    const int n = arity(op);
    const bool imm_op = op == BQ_F_LD || op == BQ_F_CONST || op == BQ_F_INRANGE || op == BQ_F_ST;
    const int idx[3] = {a, b, c};
    for (int k = 0; k < n; ++k) {
      const bool is_const = !imm_op && ((imm >> k) & 1);
      if (idx[k] >= (is_const ? P->n_const : P->n_regs)) return BQ_EINVAL;
    }
    if (!imm_op && (imm >> n) != 0) return BQ_EINVAL;   // flags only for the operands used
    if (op == BQ_F_LD && (b >= P->n_in || c >= P->n_const)) return BQ_EINVAL;
    if (op == BQ_F_CONST && (imm < 0 || imm >= P->n_const)) return BQ_EINVAL;
    if (op == BQ_F_ST && (imm < 0 || imm >= P->n_out)) return BQ_EINVAL;
  }
  static_assert(sizeof(bq_fused_program) <= 4000, "the program travels as a kernel argument (4 KiB)");
  if (S == 0 || T == 0 || P->n_ins == 0) return BQ_OK;
  const int nbt = (int)((T + FU_NT - 1) / FU_NT);
  const int64_t blocks = S * nbt;
  if (blocks > 0x7fffffff) return BQ_EINVAL;
  hipLaunchKernelGGL(fused_kernel, dim3((unsigned)blocks), dim3(FU_NT), 0, (hipStream_t)stream, *P, (int)T, nbt);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
