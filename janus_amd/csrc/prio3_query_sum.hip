// prio3_query_sum.hip -- the helper FLP query + decide + prepare message + prepare_next of
// Prio3Sum (one lane per report, MI355X gfx950).
//
// prio 0.16.2 FlpGeneric::query / decide for the Sum circuit (helper call
// site helper_initialized, aggregator.rs:2020-2042): one wire, gadget PolyEval(x^2 - x) called
// once per bit (calls K = bits), P = next_pow2(K + 1) points, validity output
// v = sum_(c=1..K) r^c p(alpha^c) for the gadget polynomial p of the proof.
//
// The generic lane kernel (k_query) runs two P-point DFTs through HBM scratch per report (the
// Lagrange basis at t, and p on the roots) and fully reduces every product: 6.3 ms per 1.25 M
// Sum(32) reports, three times the XOF.  Here both transforms stay in registers, as NPH = P/16
// phases of one 16-point DFT each (four-step split, X[NPH k + ph] = DFT16_k(y^ph)):
//   * Lagrange: u_n = t^n / P is geometric, so y^ph_n = (G_ph / P) (t alpha^ph)^n with
//     G_ph = sum_(i<NPH) (t^16 alpha^(16 ph))^i; L_c = X[(P - c) mod P] is multiplied into the
//     wire sum f(t) = L_0 seed + sum_c L_c m_(c-1) as it leaves the DFT (lazy MACs, one
//     reduction per phase);
//   * v = sum_e q_e W_e with q = p folded mod x^P - 1 and W_e = sum_(c=1..K) (r alpha^e)^c, the
//     DFT of the truncated geometric sequence r^c: y^ph_n = (r alpha^ph)^n s(n) with
//     s(n) = sum over i of (r^16 alpha^(16 ph))^i for 1 <= n + 16 i <= K -- three distinct
//     values; when 16 | K (Sum(32), Sum(64)) s is constant for n >= 1 and is applied once per
//     phase instead of per element;
//   * p(t) as 16-coefficient blocks of lazy MACs against t^0..t^15, Horner in t^16 across the
//     blocks; the truncation sum_b 2^b m_b by shift-and-add over a 160-bit accumulator.
#include <hip/hip_runtime.h>

#include "prio3_query_sum.h"

namespace {

template <int NPH, int OCC, int LEADER = 0>
__global__ __launch_bounds__(256, OCC) void k_query_sum(DevParams p, InPtrs in, Scratch sc,
                                                      OutPtrs out) {
  qsum::query_sum_body<NPH, LEADER>(p, in, sc, out, blockIdx.x * blockDim.x + threadIdx.x);
}

}  // namespace

// Prio3Sum with 8 <= bits <= 127 (P = 16 .. 128) and the engine's twiddle table
bool query_sum_takes(const DevParams& p) {
  return p.kind == PRIO3_SUM && p.es == 16 && p.arity == 1 && p.jr_len == 1 &&
         p.calls == p.meas_len && p.P >= 16 && p.P <= 128 && p.glen == 2 * p.P - 1 &&
         p.calls + 1 <= p.P;
}

bool launch_query_sum(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st,
                      bool leader) {
  if (!query_sum_takes(p) || p.n == 0) return false;
  const uint32_t blocks = (p.n + 255) / 256;
#define QS(N)                                                             \
  do {                                                                    \
    if (leader)                                                           \
      k_query_sum<N, 3, 1><<<blocks, 256, 0, st>>>(p, in, sc, out);       \
    else                                                                  \
      k_query_sum<N, 3><<<blocks, 256, 0, st>>>(p, in, sc, out);          \
    return true;                                                          \
  } while (0)
  switch (p.P) {
    case 16: QS(1);
    case 32: QS(2);
    case 64: QS(4);
    case 128: QS(8);
  }
#undef QS
  return false;
}
