// prio3_query_wide.hip -- the helper FLP query + decide for ParallelSum(Mul, C) circuits with a
// 32-, 64- or 128-point wire-polynomial domain (Prio3SumVec bits=8 length=1000 chunk 63: 127 gadget
// calls, P = 128; Prio3Histogram(256, 16): P = 32, option qwide32), EIGHT lanes per report
// (MI355X, gfx950).
//
// prio 0.16.2 FlpGeneric::query + decide, helper side of
// Prio3::prepare_init / prepare_shares_to_prepare_message; call site helper_initialized,
// aggregator.rs:2020-2042.  Same arithmetic as k_query_ps (prio3_engine.hip) -- wire 2j of call k
// carries r^(Ck+j+1) m_(Ck+j), wire 2j+1 carries m_(Ck+j) - 1/2 -- laid out for the machine:
//
// * one lane per report (k_query_ps) spends ~3 M VALU instructions per SumVec 8x1000 report
//   (two fully reduced Field128 products per element plus a multiply per truncated bit; r02j PMC:
//   SQ_INSTS_VALU 5.9e9 per 125k reports, 16.5 ms).  Here every product is a lazily reduced MAC
//   (mac128: 16 v_mad_u64_u32, no per-product reduction), the truncation is a shift-and-add Horner
//   over a 160-bit accumulator, and the gadget polynomial is never evaluated on the roots
//   (range = sum_e coef_e sigma_(e mod P), sigma from the engine's device table).
// * the 2C wire accumulators (126 for chunk 63) cannot live in one lane's VGPRs, so the C columns
//   are dealt round-robin over the 8 lanes of the report (lane l owns columns j = l mod 8, GS of
//   them per sweep).  The per-call coefficients beta_k, L_(k+1) are the same for the 8 lanes: one
//   load instruction serves all of them, and C/(8 GS) sweeps re-read them (2 sweeps at GS = 4:
//   8 KiB per report against 125 KiB of measurement share).  Lane l = report's column owner,
//   lanes 8q..8q+7 = one report, so a load of column j by the 8 owners of a wave covers eight
//   full 128-byte rows segments of [element][report] scratch.
// * the Lagrange basis at t is a four-step DFT: X[8m + l] = DFT_(P/8)(y)[m] with
//   y_n = (1/P) G_l (t w^l)^n, G_l = sum_(i<8) (t^(P/8) w8^l)^i (u_e = t^e/P is geometric, so the
//   eight-point stage collapses to the geometric sum G_l); each lane runs one P/8-point DFT in
//   registers and owns L_c for c = (P - 8m - l) mod P.
// The eight lanes of a report exchange values through the scratch rows they write (Lbuf, beta:
// written once, then read by the whole group after a vmcnt(0) wait) and through DPP/bpermute
// group sums.
#include <hip/hip_runtime.h>

#include "prio3_query_wide.h"

namespace {

template <int PQ, int LOGQ, int GS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(GS == 2 ? 3 : 2, GS == 2 ? 3 : 2))) void k_query_w(DevParams p, InPtrs in, Scratch sc,
                                                 OutPtrs out) {
  const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
  qwide::query_w_body<PQ, LOGQ, GS>(p, in, sc, out, tid >> 3, tid & 7u);
}

}  // namespace

// true if launched: ParallelSum(Mul) instances (Histogram, SumVec with bits <= 32) with P = 32, 64
// or 128 and the engine's sigma table
bool query_wide_takes(const DevParams& p) {
  if (p.es != 16 || !p.sigma_dev || (p.P != 32 && p.P != 64 && p.P != 128)) return false;
  if (p.kind != PRIO3_HISTOGRAM && p.kind != PRIO3_SUMVEC) return false;
  if (p.kind == PRIO3_SUMVEC && p.bits > 32) return false;
  return p.calls + 1 <= p.P && p.glen == 2 * p.P - 1 && p.arity == 2 * p.chunk;
}

// three wire columns per lane and sweep (within 5 % of two and four; the width without spills)
bool launch_query_wide(const DevParams& p, InPtrs in, Scratch sc, OutPtrs out, hipStream_t st) {
  if (!query_wide_takes(p) || p.n == 0 || p.P == 32) return false;
  const uint32_t blocks = (p.n + 31) / 32;
  if (p.P == 128)
    k_query_w<16, 4, 3><<<blocks, 256, 0, st>>>(p, in, sc, out);
  else
    k_query_w<8, 3, 3><<<blocks, 256, 0, st>>>(p, in, sc, out);
  return true;
}
