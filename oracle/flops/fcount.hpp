/* FP64 operation counter for the CPU oracle (TEST / MEASUREMENT INFRASTRUCTURE ONLY).
 *
 * The oracle's C sources are compiled as C++ with `double` redefined to `fdbl`, a one-member
 * struct with the size and alignment of double (so every struct, including the ur3e_model_t image
 * and the ctypes buffers, keeps its layout).  Each +, -, *, / and sqrt on an fdbl increments a
 * thread-local counter: the algorithmic FP64 operation count of the oracle's pipeline, which the
 * GPU kernels execute in the same order (bench.py's FP64 roofline).  Comparisons, fabs, copies,
 * selects and conversions are not counted. */
#ifndef UR3E_FCOUNT_HPP
#define UR3E_FCOUNT_HPP
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <stdint.h>
#include <type_traits>

extern "C" {
extern __thread unsigned long long ur3f_flops;
}

struct fdbl {
  double v;
  fdbl() = default;
  template <class T, class = typename std::enable_if<std::is_arithmetic<T>::value>::type>
  constexpr fdbl(T x) : v((double)x) {}
  template <class T, class = typename std::enable_if<std::is_arithmetic<T>::value>::type>
  explicit constexpr operator T() const { return (T)v; }
  fdbl& operator+=(fdbl o) { ++ur3f_flops; v += o.v; return *this; }
  fdbl& operator-=(fdbl o) { ++ur3f_flops; v -= o.v; return *this; }
  fdbl& operator*=(fdbl o) { ++ur3f_flops; v *= o.v; return *this; }
  fdbl& operator/=(fdbl o) { ++ur3f_flops; v /= o.v; return *this; }
};
static_assert(sizeof(fdbl) == sizeof(double) && alignof(fdbl) == alignof(double), "fdbl layout");
static inline fdbl operator+(fdbl a, fdbl b) { ++ur3f_flops; return fdbl(a.v + b.v); }
static inline fdbl operator-(fdbl a, fdbl b) { ++ur3f_flops; return fdbl(a.v - b.v); }
static inline fdbl operator*(fdbl a, fdbl b) { ++ur3f_flops; return fdbl(a.v * b.v); }
static inline fdbl operator/(fdbl a, fdbl b) { ++ur3f_flops; return fdbl(a.v / b.v); }
static inline fdbl operator-(fdbl a) { return fdbl(-a.v); }
static inline fdbl operator+(fdbl a) { return a; }
static inline bool operator<(fdbl a, fdbl b) { return a.v < b.v; }
static inline bool operator>(fdbl a, fdbl b) { return a.v > b.v; }
static inline bool operator<=(fdbl a, fdbl b) { return a.v <= b.v; }
static inline bool operator>=(fdbl a, fdbl b) { return a.v >= b.v; }
static inline bool operator==(fdbl a, fdbl b) { return a.v == b.v; }
static inline bool operator!=(fdbl a, fdbl b) { return a.v != b.v; }
static inline bool operator!(fdbl a) { return !a.v; }
static inline fdbl sqrt(fdbl a) { ++ur3f_flops; return fdbl(::sqrt(a.v)); }
static inline fdbl fabs(fdbl a) { return fdbl(::fabs(a.v)); }
static inline fdbl floor(fdbl a) { return fdbl(::floor(a.v)); }
static inline fdbl ceil(fdbl a) { return fdbl(::ceil(a.v)); }
static inline fdbl copysign(fdbl a, fdbl b) { return fdbl(::copysign(a.v, b.v)); }
static inline fdbl fmin(fdbl a, fdbl b) { return fdbl(::fmin(a.v, b.v)); }
static inline fdbl fmax(fdbl a, fdbl b) { return fdbl(::fmax(a.v, b.v)); }
static inline fdbl ldexp(fdbl a, int e) { return fdbl(::ldexp(a.v, e)); }
static inline int isnan(fdbl a) { return ::isnan(a.v); }
static inline int isinf(fdbl a) { return ::isinf(a.v); }
static inline int isfinite(fdbl a) { return ::isfinite(a.v); }
#define double fdbl
#endif
