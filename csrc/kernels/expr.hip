// K18 fused elementwise expressions (D3 column expressions: log / exp / casts / when /
// comparisons / arithmetic, e.g. ML 01:157-160 price casts, L03:79-107 log-price + exp back,
// MLE 03:51 when-label).
//
// The torch path evaluates an expression tree one operator at a time: every node is a kernel that reads
// and writes whole columns (plus a validity mask) through HBM.  Here the host compiles the tree into a
// postfix program and ONE kernel runs it per row: inputs are read once, intermediates live in a per-block
// LDS operand stack ([16 slots][256 rows] fp64 + validity bytes; the stack depth is data-independent, so
// the stack pointer is a wave-uniform scalar and every lane executes the same opcode -- no divergence), and
// the result is written once.  Null semantics follow the torch operators exactly (Spark three-valued
// logic, division / modulo by zero and log / sqrt of out-of-domain values produce nulls).
#include "common.h"

namespace {

constexpr int kExprThreads = 256;
constexpr int kExprMaxIn = 16;
constexpr int kExprStack = 16;
constexpr int kExprMaxProg = 256;

// input / output dtype codes
enum : int { DT_F64 = 0, DT_F32 = 1, DT_I32 = 2, DT_I64 = 3, DT_BOOL = 4 };

// opcodes (instruction = op | arg << 8); keep in sync with cdnaml/sql/fused.py
enum : int {
  OP_LOAD = 1, OP_CONST = 2, OP_NULL = 3,
  OP_ADD = 10, OP_SUB = 11, OP_MUL = 12, OP_DIV = 13, OP_MOD = 14, OP_POW = 15,
  OP_EQ = 20, OP_NE = 21, OP_LT = 22, OP_LE = 23, OP_GT = 24, OP_GE = 25, OP_EQNS = 26,
  OP_AND = 30, OP_OR = 31, OP_BAND = 33, OP_BOR = 34, OP_BXOR = 35, OP_NOT = 39,  // binary ops: 10..35
  OP_NEG = 40, OP_ABS = 41, OP_LN = 42, OP_LOG10 = 43, OP_LOG2 = 44, OP_LOG1P = 45, OP_EXP = 46,
  OP_EXPM1 = 47, OP_SQRT = 48, OP_FLOOR = 49, OP_CEIL = 50, OP_SIGNUM = 51, OP_SIN = 52, OP_COS = 53,
  OP_TAN = 54, OP_ROUND = 55,
  OP_TO_I32 = 60, OP_TO_I64 = 61, OP_TO_BOOL = 62, OP_TO_F32 = 63,
  OP_ISNULL = 70, OP_ISNOTNULL = 71, OP_ISNAN = 72,
  OP_CASE = 80,  // stack: ... acc_value, cond, branch_value -> acc (takes the branch where cond is true)
};

struct ExprArgs {
  const void* in[kExprMaxIn];
  const uint8_t* inv[kExprMaxIn];  // validity (nullptr = all valid)
  int indt[kExprMaxIn];
  const int* prog;
  int nprog;
  const double* consts;
  int64_t n;
  void* out;
  int outdt;
  uint8_t* outv;  // nullptr: result cannot be null
};

__device__ __forceinline__ double load_in(const ExprArgs& a, int k, int64_t r) {
  switch (a.indt[k]) {
    case DT_F64: return reinterpret_cast<const double*>(a.in[k])[r];
    case DT_F32: return (double)reinterpret_cast<const float*>(a.in[k])[r];
    case DT_I32: return (double)reinterpret_cast<const int32_t*>(a.in[k])[r];
    case DT_I64: return (double)reinterpret_cast<const int64_t*>(a.in[k])[r];
    default: return reinterpret_cast<const uint8_t*>(a.in[k])[r] ? 1.0 : 0.0;
  }
}

__global__ __launch_bounds__(kExprThreads) void expr_eval_kernel(const ExprArgs a) {
  __shared__ double sv[kExprStack][kExprThreads];
  __shared__ uint8_t sm[kExprStack][kExprThreads];
  __shared__ int sprog[kExprMaxProg];
  for (int i = threadIdx.x; i < a.nprog; i += kExprThreads) sprog[i] = a.prog[i];
  __syncthreads();
  const int t = threadIdx.x;
  for (int64_t r0 = (int64_t)blockIdx.x * kExprThreads; r0 < a.n; r0 += (int64_t)gridDim.x * kExprThreads) {
    const int64_t r = r0 + t;
    const bool live = r < a.n;
    const int64_t rr = live ? r : a.n - 1;  // idle lanes evaluate the last row (results discarded)
    int sp = 0;                             // wave-uniform
    for (int pc = 0; pc < a.nprog; ++pc) {
      const int ins = sprog[pc];
      const int op = ins & 0xFF, arg = ins >> 8;
      if (op == OP_LOAD) {
        sv[sp][t] = load_in(a, arg, rr);
        sm[sp][t] = a.inv[arg] ? a.inv[arg][rr] : (uint8_t)1;
        ++sp;
        continue;
      }
      if (op == OP_CONST || op == OP_NULL) {
        sv[sp][t] = op == OP_CONST ? a.consts[arg] : 0.0;
        sm[sp][t] = op == OP_CONST;
        ++sp;
        continue;
      }
      if (op >= OP_ADD && op <= OP_BXOR) {  // binary
        const double x = sv[sp - 2][t], y = sv[sp - 1][t];
        const uint8_t mx = sm[sp - 2][t], my = sm[sp - 1][t];
        double v = 0.0;
        uint8_t m = mx & my;
        switch (op) {
          case OP_ADD: v = x + y; break;
          case OP_SUB: v = x - y; break;
          case OP_MUL: v = x * y; break;
          case OP_DIV: v = x / (y == 0.0 ? 1.0 : y); m &= (uint8_t)(y != 0.0); break;
          case OP_MOD: v = fmod(x, y == 0.0 ? 1.0 : y); m &= (uint8_t)(y != 0.0); break;
          case OP_POW: v = pow(x, y); break;
          case OP_EQ: v = x == y; break;
          case OP_NE: v = x != y; break;
          case OP_LT: v = x < y; break;
          case OP_LE: v = x <= y; break;
          case OP_GT: v = x > y; break;
          case OP_GE: v = x >= y; break;
          case OP_EQNS: v = (mx && my && x == y) || (!mx && !my); m = 1; break;  // <=> null-safe equality
          case OP_AND: {
            const bool bx = x != 0.0, by = y != 0.0;
            m = (uint8_t)((mx && my) || (mx && !bx) || (my && !by));  // null AND false = false
            v = (bx && by && m) ? 1.0 : 0.0;
            break;
          }
          case OP_OR: {
            const bool bx = x != 0.0, by = y != 0.0;
            m = (uint8_t)((mx && my) || (mx && bx) || (my && by));    // null OR true = true
            v = ((bx || by) && m) ? 1.0 : 0.0;
            break;
          }
          case OP_BAND: v = (x != 0.0) && (y != 0.0); break;
          case OP_BOR: v = (x != 0.0) || (y != 0.0); break;
          default: v = (x != 0.0) != (y != 0.0); break;  // OP_BXOR
        }
        sv[sp - 2][t] = v;
        sm[sp - 2][t] = m;
        --sp;
        continue;
      }
      if (op == OP_CASE) {
        const double acc = sv[sp - 3][t], c = sv[sp - 2][t], bv = sv[sp - 1][t];
        const uint8_t macc = sm[sp - 3][t], mc = sm[sp - 2][t], mb = sm[sp - 1][t];
        const bool take = mc && c != 0.0;
        sv[sp - 3][t] = take ? bv : acc;
        sm[sp - 3][t] = take ? mb : macc;
        sp -= 2;
        continue;
      }
      // unary
      const double x = sv[sp - 1][t];
      uint8_t m = sm[sp - 1][t];
      double v;
      switch (op) {
        case OP_NOT: v = x == 0.0; break;
        case OP_NEG: v = -x; break;
        case OP_ABS: v = fabs(x); break;
        case OP_LN: v = log(x); m &= (uint8_t)(x > 0.0); break;
        case OP_LOG10: v = log10(x); m &= (uint8_t)(x > 0.0); break;
        case OP_LOG2: v = log2(x); m &= (uint8_t)(x > 0.0); break;
        case OP_LOG1P: v = log1p(x); m &= (uint8_t)(x > -1.0); break;
        case OP_EXP: v = exp(x); break;
        case OP_EXPM1: v = expm1(x); break;
        case OP_SQRT: v = sqrt(x); m &= (uint8_t)!(x < 0.0); break;
        case OP_FLOOR: v = floor(x); break;
        case OP_CEIL: v = ceil(x); break;
        case OP_SIGNUM: v = x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x)); break;
        case OP_SIN: v = sin(x); break;
        case OP_COS: v = cos(x); break;
        case OP_TAN: v = tan(x); break;
        case OP_ROUND: {  // HALF_UP at 10^arg (arg is the scale + 128)
          const double p = pow(10.0, (double)(arg - 128));
          v = (x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : x)) * floor(fabs(x) * p + 0.5) / p;  // torch.sign: NaN stays
          break;
        }
        case OP_TO_I32:
        case OP_TO_I64: {
          const bool bad = !isfinite(x);
          v = bad ? 0.0 : trunc(x);
          m &= (uint8_t)!bad;
          break;
        }
        case OP_TO_BOOL: v = x != 0.0; break;
        case OP_TO_F32: v = (double)(float)x; break;
        case OP_ISNULL: v = !m; m = 1; break;
        case OP_ISNOTNULL: v = m; m = 1; break;
        case OP_ISNAN: v = isnan(x) ? 1.0 : 0.0; break;
        default: v = x; break;
      }
      sv[sp - 1][t] = v;
      sm[sp - 1][t] = m;
    }
    if (live) {
      const double v = sv[0][t];
      switch (a.outdt) {
        case DT_F64: reinterpret_cast<double*>(a.out)[r] = v; break;
        case DT_F32: reinterpret_cast<float*>(a.out)[r] = (float)v; break;
        case DT_I32: reinterpret_cast<int32_t*>(a.out)[r] = (int32_t)v; break;
        case DT_I64: reinterpret_cast<int64_t*>(a.out)[r] = (int64_t)v; break;
        default: reinterpret_cast<uint8_t*>(a.out)[r] = v != 0.0; break;
      }
      if (a.outv) a.outv[r] = sm[0][t];
    }
  }
}

}  // namespace

// prog: nprog instructions (op | arg << 8), max stack depth <= 16 (host-checked); in / inv / indt: ninp inputs.
CDNA_API int cdna_expr_eval(const int* prog, int nprog, const double* consts, int ninp, const void* const* in,
                            const uint8_t* const* inv, const int* indt, int64_t n, void* out, int outdt,
                            uint8_t* outv, hipStream_t st) {
  if (n <= 0) return 0;
  if (nprog <= 0 || nprog > kExprMaxProg || ninp > kExprMaxIn) return (int)hipErrorInvalidValue;
  ExprArgs a{};
  for (int k = 0; k < ninp; ++k) {
    a.in[k] = in[k];
    a.inv[k] = inv[k];
    a.indt[k] = indt[k];
  }
  a.prog = prog;
  a.nprog = nprog;
  a.consts = consts;
  a.n = n;
  a.out = out;
  a.outdt = outdt;
  a.outv = outv;
  int64_t blocks = (n + kExprThreads - 1) / kExprThreads;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(expr_eval_kernel, dim3((unsigned)blocks), dim3(kExprThreads), 0, st, a);
  return (int)hipGetLastError();
}
