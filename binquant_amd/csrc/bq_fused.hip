// Fused element-wise programs (bq_fused_eval, include/binquant_amd.h): the
// element-wise glue between the rolling series of the strategy pipelines
//  as one launch per stage instead of one torch kernel
// per operator, each of which reads and writes a whole [S, T] fp64 panel.
//
// Mapping: a block = 256 consecutive candles of one symbol (coalesced loads /
// stores, shifted loads are offset rows of the same lines), one or two per
// thread. The
// program is wave-uniform: instructions and operand descriptors are read
// from the kernarg segment with scalar loads and dispatched by a scalar
// branch. Program registers live in LDS ([reg][thread], conflict-free,
// sized to the program's register count);
// the loads are issued together first (up to 16 in flight per thread) so a
// thread waits for HBM once, not once per operand. Arithmetic is plain IEEE
// fp64 (-ffp-contract=off: no FMA contraction), in the program's order.
// Constant operands are read from the kernarg table directly (no register).
#include "bq_device.h"
#include "binquant_amd.h"
#include "bq_fused_jit.h"

#include <string.h>

namespace bq {

constexpr int FU_SPAN = 256;   // candles per block

// The launch form of a program (translated from bq_fused_program on the
// host, once per call): every operand of every instruction is pre-resolved
// to an LDS slot — registers at r * NT + thread, constants (copied into LDS
// once per block) at a slot every lane reads — so an instruction reads its
// three operands with three independent LDS loads and one wait, no branches
// and no scalar address arithmetic.
//   code: op (6 bits) | dst slot (13) | A | B | C, operand = slot << 1 | per-lane (14 bits each)
//   aux:  LD: shift (16, signed) | operand index << 16 | fill constant << 24;
//         INRANGE: shift; ST: output index
enum : int { FK_MOV = 63 };
struct FusedLaunch {
  int32_t n_ins, n_loads, n_const, cbase;
  uint64_t code[BQ_FUSED_MAX_INS];
  int32_t aux[BQ_FUSED_MAX_INS];
  double consts[BQ_FUSED_MAX_CONST];
  bq_fused_operand in[BQ_FUSED_MAX_IN];
  bq_fused_operand out[BQ_FUSED_MAX_OUT];
};
static_assert(sizeof(FusedLaunch) <= 4000, "the program travels as a kernel argument (4 KiB)");

__device__ __forceinline__ double fused_load(const bq_fused_operand& X, int64_t sym, int ts) {
  const int64_t off = sym * X.stride_s + (int64_t)ts * X.stride_t;
  return X.dtype == BQ_F_U8 ? (double)(static_cast<const uint8_t*>(X.ptr)[off] != 0)
                            : static_cast<const double*>(X.ptr)[off];
}

// one decoded instruction over the K candles of a thread: the dispatch is
// once per instruction, the arithmetic an element-wise vector expression
template <int K>
__device__ __forceinline__ auto vec_op(int op, double __attribute__((ext_vector_type(K))) x,
                                       double __attribute__((ext_vector_type(K))) y,
                                       double __attribute__((ext_vector_type(K))) z) {
  typedef double vk __attribute__((ext_vector_type(K)));
  vk r;
  auto b = [](bool c) { return c ? 1.0 : 0.0; };
  switch (op) {
    case BQ_F_ADD: return x + y;
    case BQ_F_SUB: return x - y;
    case BQ_F_MUL: return x * y;
    case BQ_F_DIV: return x / y;
    case BQ_F_NEG: return -x;
#define BQ_EACH(expr)                          \
  _Pragma("unroll") for (int k = 0; k < K; ++k) { \
    const double u = x[k], v = y[k], w = z[k];  \
    (void)v;                                    \
    (void)w;                                    \
    r[k] = (expr);                              \
  }                                             \
  return r;
    case BQ_F_FMAX: BQ_EACH(fmax(u, v))
    case BQ_F_FMIN: BQ_EACH(fmin(u, v))
    case BQ_F_MAXIMUM: BQ_EACH((u != u || v != v) ? qnan() : (u > v ? u : v))
    case BQ_F_MINIMUM: BQ_EACH((u != u || v != v) ? qnan() : (u < v ? u : v))
    case BQ_F_GT: BQ_EACH(b(u > v))
    case BQ_F_GE: BQ_EACH(b(u >= v))
    case BQ_F_LT: BQ_EACH(b(u < v))
    case BQ_F_LE: BQ_EACH(b(u <= v))
    case BQ_F_EQ: BQ_EACH(b(u == v))
    case BQ_F_NE: BQ_EACH(b(u != v))
    case BQ_F_AND: BQ_EACH(b(u != 0.0 && v != 0.0))
    case BQ_F_OR: BQ_EACH(b(u != 0.0 || v != 0.0))
    case BQ_F_NOT: BQ_EACH(b(u == 0.0))
    case BQ_F_ABS: BQ_EACH(fabs(u))
    case BQ_F_ISNAN: BQ_EACH(b(u != u))
    case BQ_F_SQRT: BQ_EACH(sqrt(u))
    case BQ_F_LOG: BQ_EACH(log(u))
    case BQ_F_WHERE: BQ_EACH(u != 0.0 ? v : w)
#undef BQ_EACH
    default: return x;   // FK_MOV (a constant into a register)
  }
}

// K candles per thread (t = block start + k * NT + thread): one decoded
// instruction is applied to K elements, and a slot is K consecutive doubles
// in LDS (ds_read_b128 pairs).
template <int K>
__global__ __launch_bounds__(FU_SPAN / K) void fused_kernel(const FusedLaunch P, int T, int nbt) {
  constexpr int NT = FU_SPAN / K;
  constexpr int LB = K >= 4 ? 8 : 16;   // loads in flight per batch (VGPR budget)
  typedef double vk __attribute__((ext_vector_type(K)));
  extern __shared__ double fused_lds[];
  vk* R = reinterpret_cast<vk*>(fused_lds);   // [n_regs][NT] slots, then the constants
  const int tid = threadIdx.x;
  const int64_t sym = blockIdx.x / nbt;
  const int t0 = (int)(blockIdx.x % nbt) * FU_SPAN + tid;
  for (int j = tid; j < P.n_const; j += NT) R[P.cbase + j] = vk(P.consts[j]);
  auto load = [&](int ax) -> vk {
    const int sh = (int)(int16_t)(ax & 0xffff), b = (ax >> 16) & 0xff, c = (ax >> 24) & 0xff;
    vk v;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int ts = t0 + k * NT - sh;
      v[k] = (t0 + k * NT < T && ts >= 0 && ts < T) ? fused_load(P.in[b], sym, ts) : P.consts[c];
    }
    return v;
  };
  auto slot = [&](uint64_t o) -> int { return (int)(o >> 1) + ((o & 1) ? tid : 0); };

  // the load block, LB loads in flight at a time
  for (int i0 = 0; i0 < P.n_loads; i0 += LB) {
    vk lv[LB];
#pragma unroll
    for (int i = 0; i < LB; ++i)
      if (i0 + i < P.n_loads) lv[i] = load(P.aux[i0 + i]);
#pragma unroll
    for (int i = 0; i < LB; ++i)
      if (i0 + i < P.n_loads) R[(int)((P.code[i0 + i] >> 6) & 0x1fff) + tid] = lv[i];
  }
  __syncthreads();   // the constants

  for (int pc = P.n_loads; pc < P.n_ins; ++pc) {
    const uint64_t cw = P.code[pc];
    const int op = (int)(cw & 63);
    const int d = (int)((cw >> 6) & 0x1fff) + tid;
    // only the operands the op reads (arity in bits 61-62; wave-uniform
    // branch): the interpreter is LDS-bandwidth bound, and a unary or binary
    // op no longer pays for three operand reads
    const int na = (int)(cw >> 61) & 3;
    const vk x = R[slot((cw >> 19) & 0x3fff)];
    vk y = x, z = x;
    if (na >= 2) y = R[slot((cw >> 33) & 0x3fff)];
    if (na >= 3) z = R[slot((cw >> 47) & 0x3fff)];
    vk r;
    if (op == BQ_F_ST) {
      const bq_fused_operand& Y = P.out[P.aux[pc]];
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int t = t0 + k * NT;
        if (t < T) {
          const int64_t off = sym * Y.stride_s + (int64_t)t * Y.stride_t;
          if (Y.dtype == BQ_F_U8) static_cast<uint8_t*>(const_cast<void*>(Y.ptr))[off] = x[k] != 0.0;
          else static_cast<double*>(const_cast<void*>(Y.ptr))[off] = x[k];
        }
      }
      continue;
    } else if (op == BQ_F_LD) {   // a load after the block (programs with > 16 loads)
      r = load(P.aux[pc]);
    } else if (op == BQ_F_INRANGE) {
      const int sh = P.aux[pc];
#pragma unroll
      for (int k = 0; k < K; ++k) r[k] = (t0 + k * NT - sh >= 0 && t0 + k * NT - sh < T) ? 1.0 : 0.0;
    } else {
      r = vec_op<K>(op, x, y, z);
    }
    R[d] = r;
  }
}

}  // namespace bq

namespace {

int arity(int op);

// bq_fused_program (ABI form, validated) -> the launch form for NT threads
void translate(const bq_fused_program& P, int NT, bq::FusedLaunch& L) {
  memset(&L, 0, sizeof(L));
  L.n_ins = P.n_ins;
  L.n_loads = P.n_loads;
  L.n_const = P.n_const;
  L.cbase = P.n_regs * NT;
  memcpy(L.consts, P.consts, sizeof(L.consts));
  memcpy(L.in, P.in, sizeof(L.in));
  memcpy(L.out, P.out, sizeof(L.out));
  auto reg_opd = [&](uint64_t r) -> uint64_t { return ((uint64_t)(r * NT) << 1) | 1ull; };
  auto const_opd = [&](uint64_t j) -> uint64_t { return (uint64_t)(L.cbase + j) << 1; };
  const uint64_t none = const_opd(0);   // harmless slot for unused operands
  for (int pc = 0; pc < P.n_ins; ++pc) {
    const uint64_t in = P.ins[pc];
    int op = (int)(in & 0xff);
    const uint64_t d = (in >> 8) & 0xff, a = (in >> 16) & 0xff, b = (in >> 24) & 0xff, c = (in >> 32) & 0xff;
    const int64_t imm = (int64_t)in >> 40;
    uint64_t A = none, B = none, C = none;
    int32_t aux = 0;
    switch (op) {
      case BQ_F_LD: aux = (int32_t)((imm & 0xffff) | (int64_t)(b << 16) | (int64_t)(c << 24)); break;
      case BQ_F_CONST: op = bq::FK_MOV; A = const_opd((uint64_t)imm); break;
      case BQ_F_INRANGE: aux = (int32_t)imm; break;
      case BQ_F_ST: A = reg_opd(a); aux = (int32_t)imm; break;
      default: {
        const uint64_t ops[3] = {a, b, c};
        uint64_t* dst[3] = {&A, &B, &C};
        const int n = op == BQ_F_WHERE ? 3 : (op == BQ_F_NOT || (op >= BQ_F_ABS && op <= BQ_F_LOG)) ? 1 : 2;
        for (int k = 0; k < n; ++k) *dst[k] = ((imm >> k) & 1) ? const_opd(ops[k]) : reg_opd(ops[k]);
      }
    }
    const uint64_t na = op == bq::FK_MOV ? 1 : (uint64_t)arity(op);
    L.code[pc] = (uint64_t)op | ((uint64_t)(d * NT) << 6) | (A << 19) | (B << 33) | (C << 47) | (na << 61);
    L.aux[pc] = aux;
  }
}

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

namespace bq {

int fused_validate(const bq_fused_program& P) {
  if (P.n_ins < 0 || P.n_ins > BQ_FUSED_MAX_INS || P.n_loads < 0 || P.n_loads > BQ_FUSED_MAX_LOADS ||
      P.n_loads > P.n_ins || P.n_regs < 0 || P.n_regs > BQ_FUSED_MAX_REGS || P.n_in < 0 ||
      P.n_in > BQ_FUSED_MAX_IN || P.n_out < 0 || P.n_out > BQ_FUSED_MAX_OUT || P.n_const < 0 ||
      P.n_const > BQ_FUSED_MAX_CONST)
    return BQ_EINVAL;
  for (int i = 0; i < P.n_in; ++i)
    if (!operand_ok(P.in[i])) return BQ_EINVAL;
  for (int i = 0; i < P.n_out; ++i)
    if (!operand_ok(P.out[i])) return BQ_EINVAL;
  for (int pc = 0; pc < P.n_ins; ++pc) {
    const uint64_t in = P.ins[pc];
    const int op = (int)(in & 0xff);
    const int d = (int)((in >> 8) & 0xff), a = (int)((in >> 16) & 0xff), b = (int)((in >> 24) & 0xff),
              c = (int)((in >> 32) & 0xff);
    const int64_t imm = (int64_t)in >> 40;
    if (op < BQ_F_LD || op > BQ_F_ST) return BQ_EINVAL;
    if (pc < P.n_loads && op != BQ_F_LD) return BQ_EINVAL;   // the load block comes first
    if (op != BQ_F_ST && d >= P.n_regs) return BQ_EINVAL;
    const int n = arity(op);
    const bool imm_op = op == BQ_F_LD || op == BQ_F_CONST || op == BQ_F_INRANGE || op == BQ_F_ST;
    const int idx[3] = {a, b, c};
    for (int k = 0; k < n; ++k) {
      const bool is_const = !imm_op && ((imm >> k) & 1);
      if (idx[k] >= (is_const ? P.n_const : P.n_regs)) return BQ_EINVAL;
    }
    if (!imm_op && (imm >> n) != 0) return BQ_EINVAL;   // flags only for the operands used
    if (op == BQ_F_LD && (b >= P.n_in || c >= P.n_const)) return BQ_EINVAL;
    if (op == BQ_F_CONST && (imm < 0 || imm >= P.n_const)) return BQ_EINVAL;
    if (op == BQ_F_ST && (imm < 0 || imm >= P.n_out)) return BQ_EINVAL;
  }
  return BQ_OK;
}

}  // namespace bq

extern "C" {

int bq_fused_eval(const bq_fused_program* P, int64_t S, int64_t T, void* stream) {
  using namespace bq;
  if (!P || S < 0 || T < 0 || T > 0x7fffffff) return BQ_EINVAL;
  if (fused_validate(*P) != BQ_OK) return BQ_EINVAL;
  if (S == 0 || T == 0 || P->n_ins == 0) return BQ_OK;
  if (fused_native_enabled()) return fused_native_eval(*P, S, T, (hipStream_t)stream);
  const int nbt = (int)((T + FU_SPAN - 1) / FU_SPAN);
  const int64_t blocks = S * nbt;
  if (blocks > 0x7fffffff) return BQ_EINVAL;
  const size_t lds = ((size_t)P->n_regs * FU_SPAN + (size_t)(P->n_const + 1) * 2) * sizeof(double);
  if (P->n_regs * FU_SPAN + P->n_const + 1 >= (1 << 13)) return BQ_EINVAL;   // slot field width
  FusedLaunch L;
  // candles per thread: more amortise the decode over more elements, but a
  // program register costs K * 512 bytes of LDS per wave; keep >= 8 waves per
  // CU (160 KiB), and one candle per thread on short rows (live frames of a
  // few hundred bars) so no thread idles on the tail
  const int K = T < 4 * FU_SPAN ? 1 : P->n_regs <= 10 ? 4 : P->n_regs <= 20 ? 2 : 1;
  translate(*P, FU_SPAN / K, L);
  hipStream_t st = (hipStream_t)stream;
  if (K == 4)
    hipLaunchKernelGGL(fused_kernel<4>, dim3((unsigned)blocks), dim3(FU_SPAN / 4), lds, st, L, (int)T, nbt);
  else if (K == 2)
    hipLaunchKernelGGL(fused_kernel<2>, dim3((unsigned)blocks), dim3(FU_SPAN / 2), lds, st, L, (int)T, nbt);
  else
    hipLaunchKernelGGL(fused_kernel<1>, dim3((unsigned)blocks), dim3(FU_SPAN), lds, st, L, (int)T, nbt);
  return hipGetLastError() == hipSuccess ? BQ_OK : BQ_EHIP;
}

}  // extern "C"
