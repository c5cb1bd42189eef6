// ecdh_a3.h -- ECDH on a short-Weierstrass curve with a = -3 over a field F (p521_device.h's
// Field), for the NIST-curve DHKEMs of the HPKE opener (hpke.hip).  The algorithm is the one
// p256_device.h's ecdh runs with its generated-asm field: validate the peer point, build the
// affine odd multiples P, 3P, .., 15P (one inversion by Montgomery's trick), then a fixed signed
// window (w = 4) over the host-recoded server key -- the same key in every lane, so every lane
// runs the same instruction stream and reads the table at a wave-uniform index.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#ifndef DEV
#define DEV __device__ __forceinline__
#endif

namespace ecdh_a3 {

template <class F>
struct jac {
  typename F::T X, Y, Z;
};

// dbl-2001-b (a = -3), Z3 = 2 Y Z
template <class F>
DEV jac<F> dbl(const jac<F>& P) {
  typedef typename F::T T;
  const T delta = F::sqr(P.Z), gamma = F::sqr(P.Y), beta = F::mul(P.X, gamma);
  const T alpha = F::mul_small(F::mul(F::sub(P.X, delta), F::add(P.X, delta)), 3);
  const T b4 = F::mul_small(beta, 4);
  jac<F> R;
  R.X = F::sub(F::sqr(alpha), F::add(b4, b4));
  const T yz = F::mul(P.Y, P.Z);
  R.Z = F::add(yz, yz);
  R.Y = F::sub(F::mul(alpha, F::sub(b4, R.X)), F::mul_small(F::sqr(gamma), 8));
  return R;
}

// madd-2007-bl: P (Jacobian) + (x2, y2) (affine), P != +-(x2, y2), P not at infinity
template <class F>
DEV jac<F> madd(const jac<F>& P, const typename F::T& x2, const typename F::T& y2) {
  typedef typename F::T T;
  const T Z1Z1 = F::sqr(P.Z);
  const T U2 = F::mul(x2, Z1Z1), S2 = F::mul(y2, F::mul(P.Z, Z1Z1));
  const T H = F::sub(U2, P.X), HH = F::sqr(H);
  const T I = F::mul_small(HH, 4), J = F::mul(H, I);
  const T s = F::sub(S2, P.Y), rr = F::add(s, s), V = F::mul(P.X, I);
  jac<F> R;
  R.X = F::sub(F::sub(F::sqr(rr), J), F::add(V, V));
  const T yj = F::mul(P.Y, J);
  R.Y = F::sub(F::mul(rr, F::sub(V, R.X)), F::add(yj, yj));
  const T zh = F::mul(P.Z, H);
  R.Z = F::add(zh, zh);
  return R;
}

// The four doublings of a window as one out-of-line call whose body inlines the field products
// of FD (P-521: the 18-limb operands exceed the calling convention's argument registers, so
// every out-of-line product passes them through scratch; here only R does, once per window)
template <class FD>
__device__ __noinline__ void dbl4(jac<FD>& R) {
  jac<FD> Q = R;
#pragma unroll 1
  for (int j = 0; j < 4; j++) Q = dbl<FD>(Q);
  R = Q;
}

// DH(sk, pkE) for an uncompressed SEC 1 point enc = 0x04 || X || Y (1 + 2 kBytes bytes): validates
// the point (prefix, canonical coordinates, y^2 = x^3 - 3x + b) and writes the shared
// x-coordinate's kBytes big-endian bytes.  dig: NDIG signed odd digits in [-15, 15] of the
// recoded key k' (k' = sk or n - sk, whichever is odd; top digit in [1, 15]), low digit first.
// As in p256_device.h, the additions meet the doubling case only at the last window (k' close
// to n), where the doubled point, computed beside the addition for every key, is the sum.
template <class F, int NDIG, class FD = F>
DEV bool ecdh(const int8_t* dig, const uint8_t* enc, uint8_t* dh_be) {
  typedef typename F::T T;
  constexpr int NB = F::kBytes;
  T x, y;
  bool ok = enc[0] == 0x04;
  ok = F::from_be(enc + 1, x) && ok;
  ok = F::from_be(enc + 1 + NB, y) && ok;
  const T rhs = F::add(F::sub(F::mul(F::sqr(x), x), F::mul_small(x, 3)), F::b());
  ok = ok && F::eq(F::sqr(y), rhs);
  T tab[8][2], zz[8], pz[8];  // (2i+1)P: affine after the inversion; Z values; prefix products
  tab[0][0] = x;
  tab[0][1] = y;
  {
    const T ny = F::neg(y);
    auto put = [&](int k, const jac<F>& Q) {
      tab[k][0] = Q.X;
      tab[k][1] = Q.Y;
      zz[k] = Q.Z;
    };
    const jac<F> P2 = dbl<F>(jac<F>{x, y, F::one()});
    const jac<F> P3 = madd<F>(P2, x, y);
    put(1, P3);
    const jac<F> P12 = dbl<F>(dbl<F>(P3));
    put(5, madd<F>(P12, x, ny));  // 11P
    put(6, madd<F>(P12, x, y));   // 13P
    const jac<F> P4 = dbl<F>(P2);
    put(2, madd<F>(P4, x, y));    // 5P
    const jac<F> P8 = dbl<F>(P4);
    put(3, madd<F>(P8, x, ny));   // 7P
    put(4, madd<F>(P8, x, y));    // 9P
    put(7, madd<F>(dbl<F>(P8), x, ny));  // 15P
  }
  {  // Montgomery's trick: one inversion for the seven Z
    T acc = zz[1];
    pz[1] = acc;
#pragma unroll 1
    for (int k = 2; k < 8; k++) {
      acc = F::mul(acc, zz[k]);
      pz[k] = acc;
    }
    T ia = F::inv(acc);
#pragma unroll 1
    for (int k = 7; k >= 1; k--) {
      T zi = ia;
      if (k > 1) {
        zi = F::mul(ia, pz[k - 1]);
        ia = F::mul(ia, zz[k]);
      }
      const T zi2 = F::sqr(zi);
      tab[k][0] = F::mul(tab[k][0], zi2);
      tab[k][1] = F::mul(tab[k][1], F::mul(zi2, zi));
    }
  }
  auto pick = [&](int d, T& tx, T& ty) {
    const int a = (d < 0 ? -d : d) >> 1;
    tx = tab[a][0];
    ty = tab[a][1];
    const T nyy = F::neg(ty);
    if (d < 0) ty = nyy;
  };
  jac<F> R;
  pick(dig[NDIG - 1], R.X, R.Y);
  R.Z = F::one();
  auto dbl_w = [&](jac<F>& Q) {
    if constexpr (std::is_same<F, FD>::value) {
#pragma unroll 1
      for (int j = 0; j < 4; j++) Q = dbl<F>(Q);
    } else {
      jac<FD> q{Q.X, Q.Y, Q.Z};
      dbl4<FD>(q);
      Q = jac<F>{q.X, q.Y, q.Z};
    }
  };
#pragma unroll 1
  for (int i = NDIG - 2; i >= 1; i--) {
    dbl_w(R);
    T tx, ty;
    pick(dig[i], tx, ty);
    R = madd<F>(R, tx, ty);  // products out of line (inlined: 256+ VGPRs, 5.99 vs 6.88 M/s)
  }
  dbl_w(R);
  {
    T tx, ty;
    pick(dig[0], tx, ty);
    const jac<F> D = dbl<F>(R);
    const jac<F> S = madd<F>(R, tx, ty);
    R = F::is_zero(S.Z) ? D : S;
  }
  ok = ok && !F::is_zero(R.Z);
  const T zi = F::inv(R.Z);
  F::to_be(F::mul(R.X, F::sqr(zi)), dh_be);
  return ok;
}

}  // namespace ecdh_a3
