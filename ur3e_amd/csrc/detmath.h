/*
 * detmath.h — deterministic FP64 transcendental functions for the UR3e step
 * path, identical bit-for-bit on the host (gcc, x86-64 SSE2) and on gfx950.
 *
 * Why: the hot path feeds sin/cos (forward kinematics, quaternion
 * integration, scipy-style rotation vectors in pid_task_ctrl) back into a
 * chaotic contact simulation.  libm and ROCm's OCML differ in the last ulp, so
 * the GPU kernels and the CPU oracle both use these implementations, compiled
 * with -ffp-contract=off.  Accuracy vs. glibc is checked in
 * tests/test_detmath.py (≤ 2 ulp on the tested ranges).
 *
 * Algorithms: fdlibm (Sun Microsystems, 1993) kernel polynomials with a
 * 3-term Cody–Waite reduction (|x| < 2^19·π/2), exp via ln2 reduction and the
 * fdlibm rational kernel, atan via the fdlibm 4-interval reduction.
 *
 * C99-compatible: the oracle (plain C) includes this header too.
 */
#ifndef UR3E_DETMATH_H
#define UR3E_DETMATH_H

#if defined(__HIPCC__)
#define UR3E_HD __host__ __device__ static inline
#else
#define UR3E_HD static inline
#endif

#include <math.h>

/* ---- sin / cos ---------------------------------------------------------- */
UR3E_HD double ur3e_ksin(double x) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x;
  double v = z * x;
  double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
  return x + v * (S1 + z * r);
}

UR3E_HD double ur3e_kcos(double x) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x;
  double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
  double ax = x < 0 ? -x : x;
  if (ax < 0.3) return 1.0 - (0.5 * z - z * r);
  double qx;
  if (ax > 0.78125) {
    qx = 0.28125;
  } else { /* fdlibm INSERT_WORDS(qx, ix - 0x00200000, 0): |x|/4, low word cleared */
    union { double d; unsigned long long u; } t;
    t.d = ax * 0.25;
    t.u &= 0xFFFFFFFF00000000ULL;
    qx = t.d;
  }
  double hz = 0.5 * z - qx;
  double a = 1.0 - qx;
  return a - (hz - z * r);
}

/* reduce x to r in [-pi/4, pi/4], returns quadrant n */
UR3E_HD int ur3e_rem_pio2(double x, double* r) {
  const double invpio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;
  const double pio2_2 = 6.07710050630396597660e-11;
  const double pio2_3 = 2.02226624871116645580e-21;
  double fn = floor(x * invpio2 + 0.5);
  double y = x - fn * pio2_1;
  y = y - fn * pio2_2;
  y = y - fn * pio2_3;
  *r = y;
  long long n = (long long)fn;
  return (int)(n & 3);
}

UR3E_HD double ur3e_sin(double x) {
  double r;
  int n = ur3e_rem_pio2(x, &r);
  switch (n) {
    case 0: return ur3e_ksin(r);
    case 1: return ur3e_kcos(r);
    case 2: return -ur3e_ksin(r);
    default: return -ur3e_kcos(r);
  }
}

UR3E_HD double ur3e_cos(double x) {
  double r;
  int n = ur3e_rem_pio2(x, &r);
  switch (n) {
    case 0: return ur3e_kcos(r);
    case 1: return -ur3e_ksin(r);
    case 2: return -ur3e_kcos(r);
    default: return ur3e_ksin(r);
  }
}

/* ---- exp ---------------------------------------------------------------- */
UR3E_HD double ur3e_exp(double x) {
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00;
  if (x != x) return x;
  if (x > 709.78) return HUGE_VAL;
  if (x < -745.2) return 0.0;
  double k = floor(x * invln2 + 0.5);
  double hi = x - k * ln2HI;
  double lo = k * ln2LO;
  double r = hi - lo;
  double t = r * r;
  double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
  double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  return ldexp(y, (int)k);
}

UR3E_HD double ur3e_tanh(double x) {
  double ax = x < 0 ? -x : x;
  double t;
  if (ax > 22.0) {
    t = 1.0;
  } else {
    double e = ur3e_exp(2.0 * ax);
    t = 1.0 - 2.0 / (e + 1.0);
  }
  return x < 0 ? -t : t;
}

/* ---- atan / atan2 ------------------------------------------------------- */
UR3E_HD double ur3e_atan(double x) {
  const double atanhi0 = 4.63647609000806093515e-01, atanhi1 = 7.85398163397448278999e-01,
               atanhi2 = 9.82793723247329054082e-01, atanhi3 = 1.57079632679489655800e+00;
  const double atanlo0 = 2.26987774529616870924e-17, atanlo1 = 3.06161699786838301793e-17,
               atanlo2 = 1.39033110312309984516e-17, atanlo3 = 6.12323399573676603587e-17;
  const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
               aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
               aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
               aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
               aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
               aT10 = 1.62858201153657823623e-02;
  if (x != x) return x;
  double sgn = x < 0 ? -1.0 : 1.0;
  double ax = x < 0 ? -x : x;
  int id;
  double hi = 0.0, lo = 0.0;
  if (ax >= 4.3452e+19) return sgn * (atanhi3 + atanlo3);
  if (ax < 0.4375) {
    id = -1;
  } else if (ax < 1.1875) {
    if (ax < 0.6875) {
      id = 0;
      ax = (2.0 * ax - 1.0) / (2.0 + ax);
    } else {
      id = 1;
      ax = (ax - 1.0) / (ax + 1.0);
    }
  } else {
    if (ax < 2.4375) {
      id = 2;
      ax = (ax - 1.5) / (1.0 + 1.5 * ax);
    } else {
      id = 3;
      ax = -1.0 / ax;
    }
  }
  double z = ax * ax;
  double w = z * z;
  double s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  double s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return sgn * (ax - ax * (s1 + s2));
  if (id == 0) { hi = atanhi0; lo = atanlo0; }
  else if (id == 1) { hi = atanhi1; lo = atanlo1; }
  else if (id == 2) { hi = atanhi2; lo = atanlo2; }
  else { hi = atanhi3; lo = atanlo3; }
  double zz = hi - ((ax * (s1 + s2) - lo) - ax);
  return sgn * zz;
}

/* atan2(y, x) for the y >= 0 uses on this path (rotation angles); general signs handled */
UR3E_HD double ur3e_atan2(double y, double x) {
  const double pi = 3.1415926535897931160e+00, pi_lo = 1.2246467991473531772e-16;
  const double pio2 = 1.5707963267948965580e+00;
  if (x != x || y != y) return x + y;
  if (y == 0.0) {
    if (x >= 0.0 && !(x == 0.0 && 1.0 / x < 0)) return y;
    return (1.0 / y < 0 || y < 0) ? -pi : pi;
  }
  if (x == 0.0) return y > 0 ? pio2 : -pio2;
  double a = ur3e_atan((y < 0 ? -y : y) / (x < 0 ? -x : x));
  if (x > 0) return y > 0 ? a : -a;
  double r = pi - (a - pi_lo);
  return y > 0 ? r : -r;
}

#endif /* UR3E_DETMATH_H */
