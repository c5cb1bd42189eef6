// prio3_wide.h -- building blocks of the eight-lanes-per-report FLP query kernels
// (prio3_query_wide.hip: ParallelSum(Mul) on 64/128-point domains; prio3_fpvec.hip: the FPVec
// two-gadget query).  Lanes 8q..8q+7 of a wave serve one report; "group" below is those 8 lanes.
#pragma once
#include "prio3_device.h"
#include "prio3_common.h"

namespace wide {

typedef Fp128 F;
typedef f128 T;

DEV T shfl_xor128(const T& x, int m) {
  return mk128((uint32_t)__shfl_xor((int)x.w[0], m), (uint32_t)__shfl_xor((int)x.w[1], m),
               (uint32_t)__shfl_xor((int)x.w[2], m), (uint32_t)__shfl_xor((int)x.w[3], m));
}
DEV T shfl128(const T& x, int src) {
  return mk128((uint32_t)__shfl((int)x.w[0], src), (uint32_t)__shfl((int)x.w[1], src),
               (uint32_t)__shfl((int)x.w[2], src), (uint32_t)__shfl((int)x.w[3], src));
}
// sum over the 8 lanes of a report (every lane gets the total)
DEV T group_sum(T x) {
  x = F::add(x, shfl_xor128(x, 1));
  x = F::add(x, shfl_xor128(x, 2));
  return F::add(x, shfl_xor128(x, 4));
}
DEV int group_or(int v) {
  v |= __shfl_xor(v, 1);
  v |= __shfl_xor(v, 2);
  return v | __shfl_xor(v, 4);
}
// a^l for a lane-dependent l < 8, from a, a^2, a^4 (no dynamic register indexing)
DEV T lane_pow(const T& a1, const T& a2, const T& a4, uint32_t l) {
  const T one = F::one();
  const T x = F::sel(l & 1u, a1, one);
  return F::mul(F::mul(x, F::sel(l & 2u, a2, one)), F::sel(l & 4u, a4, one));
}
// a <- 2a + m over a 160-bit accumulator (no reduction; < 2^160 for at most 32 steps)
DEV void horner2(sum128& a, const T& m) {
  a.w[4] = __builtin_amdgcn_alignbit(a.w[4], a.w[3], 31);
  a.w[3] = __builtin_amdgcn_alignbit(a.w[3], a.w[2], 31);
  a.w[2] = __builtin_amdgcn_alignbit(a.w[2], a.w[1], 31);
  a.w[1] = __builtin_amdgcn_alignbit(a.w[1], a.w[0], 31);
  a.w[0] <<= 1;
  sum_add(a, m);
}
// one dwordx4 load from a clamped (always in-bounds) row, zeroed by mask when invalid
DEV T ldm(const void* base, uint32_t row, bool valid, size_t ld, uint32_t r) {
  const uint32_t msk = valid ? 0xffffffffu : 0u;
  const uint4 v = ((const uint4*)base)[(size_t)(valid ? row : 0u) * ld + r];
  return mk128(v.x & msk, v.y & msk, v.z & msk, v.w & msk);
}
DEV T sqr_n(T x, int n) {
  for (int i = 0; i < n; i++) x = F::mul(x, x);
  return x;
}
// 1 + z + ... + z^7
DEV T geo8(const T& z) {
  const T one = F::one();
  T g = F::add(z, one);
#pragma unroll
  for (int i = 0; i < 6; i++) g = F::add(F::mul(g, z), one);
  return g;
}

// DFT_N (N <= 16) of the geometric sequence c q^n, n < N, in registers: x[m] = sum_n c q^n w^(nm),
// w a principal N-th root (radix-2 DIT on the bit-reversed input, prio fft.rs butterfly order
// irrelevant here: the DFT is exact).
template <int N, int LOGN>
DEV void geo_dft_reg(T c, const T& q, const T& w, T (&x)[N]) {
  T tw[N / 2 > 0 ? N / 2 : 1];
  tw[0] = F::one();
#pragma unroll
  for (int i = 1; i < N / 2; i++) tw[i] = F::mul(tw[i - 1], w);
#pragma unroll
  for (int n = 0; n < N; n++) {
    x[LOGN ? (__builtin_bitreverse32(n) >> (32 - LOGN)) : 0] = c;
    if (n + 1 < N) c = F::mul(c, q);
  }
#pragma unroll
  for (int l = 1; l <= LOGN; l++) {
    const int half = 1 << (l - 1);
#pragma unroll
    for (int i = 0; i < half; i++) {
#pragma unroll
      for (int j = i; j < N; j += 2 * half) {
        const T u = x[j];
        const T v = i == 0 ? x[j + half] : F::mul(tw[i * (N >> l)], x[j + half]);
        x[j] = F::add(u, v);
        x[j + half] = F::sub(u, v);
      }
    }
  }
}
template <int N, int LOGN, class Emit>
DEV void geo_dft_emit(const T& c, const T& q, const T& w, Emit&& emit) {
  T x[N];
  geo_dft_reg<N, LOGN>(c, q, w, x);
#pragma unroll
  for (int m = 0; m < N; m++) emit((uint32_t)m, x[m]);
}
template <class Emit>
DEV void geo_dft_small(uint32_t logn, const T& c, const T& q, const T& w, Emit&& emit) {
  switch (logn) {  // wave-uniform
    case 0: emit(0u, c); break;
    case 1: geo_dft_emit<2, 1>(c, q, w, emit); break;
    case 2: geo_dft_emit<4, 2>(c, q, w, emit); break;
    case 3: geo_dft_emit<8, 3>(c, q, w, emit); break;
    default: geo_dft_emit<16, 4>(c, q, w, emit); break;
  }
}

// The Lagrange basis of the P-th roots at t, spread over the group: lane l gets
// X[i] = (1/P) sum_(e<P) t^e alpha_P^(e i) for i = l mod 8 (P >= 8), emitted as emit(i, X[i]);
// L_c(t) = X[(P - c) mod P] (k_query_ps).  Four-step on the geometric input (see
// prio3_query_wide.hip): X[8m + l] = DFT_(P/8)(y)[m], y_n = (G_l / P) (t w^l)^n,
// G_l = sum_(i<8) (t^(P/8) w8^l)^i; a second split of the same kind when P/8 > 16.  P < 8:
// lanes l < P evaluate X[l] directly.  roots(k) = principal 2^k-th root.
template <class Emit>
DEV void lagrange_group(const DevParams& p, uint32_t logP, const T& invP, const T& t, uint32_t l,
                        Emit&& emit) {
  auto root = [&](uint32_t k) { return F::from_words(p.roots128[k]); };
  const T one = F::one();
  if (logP < 3) {
    const uint32_t P = 1u << logP;
    if (l < P) {  // direct: sum_e t^e w^(e l) / P
      const T wl = lane_pow(root(logP), F::mul(root(logP), root(logP)), one, l);  // l < 4
      const T q = F::mul(t, wl);
      T acc = F::zero(), pw = one;
      for (uint32_t e = 0; e < P; e++) {
        acc = F::add(acc, pw);
        pw = F::mul(pw, q);
      }
      emit(l, F::mul(acc, invP));
    }
    return;
  }
  const uint32_t logN = logP - 3;                      // N = P/8 per lane
  const T wP = root(logP), wP2 = F::mul(wP, wP), wP4 = F::mul(wP2, wP2);
  const T w8 = root(3), w82 = F::mul(w8, w8), w84 = F::mul(w82, w82);
  const T tN = sqr_n(t, (int)logN);                    // t^(P/8)
  const T c = F::mul(geo8(F::mul(tN, lane_pow(w8, w82, w84, l))), invP);
  const T q = F::mul(t, lane_pow(wP, wP2, wP4, l));    // t w_P^l
  if (logN <= 4) {
    geo_dft_small(logN, c, q, root(logN), [&](uint32_t m, const T& v) { emit(8 * m + l, v); });
    return;
  }
  // N = 8 x N2: Y[8 m2 + l2] = DFT_N2(c G'_l2 (q w_N^l2)^n)[m2], G'_l2 = sum_i (q^N2 w8^l2)^i
  const uint32_t logN2 = logN - 3;
  const T wN = root(logN);
  const T qN2 = sqr_n(q, (int)logN2);
  T wNl = one, w8l = one;
  for (uint32_t l2 = 0; l2 < 8; l2++) {
    const T c2 = F::mul(c, geo8(F::mul(qN2, w8l)));
    geo_dft_small(logN2, c2, F::mul(q, wNl), root(logN2),
                  [&](uint32_t m2, const T& v) { emit(8 * (8 * m2 + l2) + l, v); });
    wNl = F::mul(wNl, wN);
    w8l = F::mul(w8l, w8);
  }
}

}  // namespace wide
