// Double-double arithmetic (host + device) for the extended-precision scalars EIGSOL_DD / EIGSOL_CDD.
//
// The reference instantiates every solver for long double and std::complex<long double>
// (ScalarConcept, src/core/types.hpp:28-30); with g++ on x86-64 that is the x87 80-bit format, a
// 64-bit significand.  gfx950 has no 80-bit arithmetic, so those scalars are carried as
// double-double values: the unevaluated sum hi + lo of two doubles with |lo| <= ulp(hi) / 2, a
// 106-bit significand.  Every finite x87 value inside the double exponent range converts exactly
// (hi = the value rounded to double, lo = the remainder, which has at most 11 significant bits).
//
// The operations are the classical error-free transformations (Dekker / Knuth two-sum, two-product
// by fused multiply-add) and the "accurate" double-double sum; relative error of +, -, * and / is a
// small multiple of 2^-104, against 2^-64 for the x87 operations they replace.
#pragma once

#include <cmath>

#ifndef EIGSOL_HD
#define EIGSOL_HD __host__ __device__ inline
#endif
// The error-free transformations need every sum and product rounded on its own: HIP compiles with
// contraction on, and a product fused into the following sum (quick_two_sum after two_prod becomes
// fma(a, b, e)) silently drops the low half.  Every double-double body below opens with this.
#define EIGSOL_EXACT _Pragma("clang fp contract(off)")

namespace eigsol {

struct alignas(16) dd {
    double hi, lo;
};
struct alignas(32) cdd {
    dd re, im;
};

EIGSOL_HD dd dd_from(double a) { EIGSOL_EXACT return dd{a, 0.0}; }

// s + e = a + b exactly (no ordering requirement)
EIGSOL_HD dd two_sum(double a, double b) {
    EIGSOL_EXACT
    const double s = a + b;
    const double bb = s - a;
    const double e = (a - (s - bb)) + (b - bb);
    return dd{s, e};
}
// s + e = a + b exactly, for |a| >= |b| (or a == 0)
EIGSOL_HD dd quick_two_sum(double a, double b) {
    EIGSOL_EXACT
    const double s = a + b;
    const double e = b - (s - a);
    return dd{s, e};
}
// p + e = a * b exactly (fma keeps the low half of the product)
EIGSOL_HD dd two_prod(double a, double b) {
    EIGSOL_EXACT
    const double p = a * b;
    const double e = std::fma(a, b, -p);
    return dd{p, e};
}

EIGSOL_HD dd dd_neg(dd a) { EIGSOL_EXACT return dd{-a.hi, -a.lo}; }

// accurate double-double sum (both low parts enter the error term)
EIGSOL_HD dd dd_add(dd a, dd b) {
    EIGSOL_EXACT
    dd s = two_sum(a.hi, b.hi);
    const dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return quick_two_sum(s.hi, s.lo);
}
EIGSOL_HD dd dd_sub(dd a, dd b) { EIGSOL_EXACT return dd_add(a, dd_neg(b)); }
EIGSOL_HD dd dd_add_d(dd a, double b) {
    EIGSOL_EXACT
    dd s = two_sum(a.hi, b);
    s.lo += a.lo;
    return quick_two_sum(s.hi, s.lo);
}

EIGSOL_HD dd dd_mul(dd a, dd b) {
    EIGSOL_EXACT
    dd p = two_prod(a.hi, b.hi);
    p.lo = std::fma(a.hi, b.lo, std::fma(a.lo, b.hi, p.lo));
    return quick_two_sum(p.hi, p.lo);
}
EIGSOL_HD dd dd_mul_d(dd a, double b) {
    EIGSOL_EXACT
    dd p = two_prod(a.hi, b);
    p.lo = std::fma(a.lo, b, p.lo);
    return quick_two_sum(p.hi, p.lo);
}

// a / b: three quotient digits (long division), correctly rounded to ~2^-104
EIGSOL_HD dd dd_div(dd a, dd b) {
    EIGSOL_EXACT
    const double q1 = a.hi / b.hi;
    dd r = dd_sub(a, dd_mul_d(b, q1));
    const double q2 = r.hi / b.hi;
    r = dd_sub(r, dd_mul_d(b, q2));
    const double q3 = r.hi / b.hi;
    return dd_add_d(quick_two_sum(q1, q2), q3);
}

// sqrt(a), a >= 0: one Newton step on the double square root (Karp's trick)
EIGSOL_HD dd dd_sqrt(dd a) {
    EIGSOL_EXACT
    if (a.hi <= 0.0) return dd{a.hi == 0.0 ? 0.0 : std::sqrt(a.hi), 0.0};   // 0, or NaN for a < 0
    const double x = 1.0 / std::sqrt(a.hi);
    const double ax = a.hi * x;
    const dd d = dd_sub(a, two_prod(ax, ax));
    return dd_add_d(dd{ax, 0.0}, d.hi * (x * 0.5));
}

EIGSOL_HD bool dd_is_zero(dd a) { return a.hi == 0.0; }   // normalised: lo == 0 whenever hi == 0
EIGSOL_HD dd dd_abs(dd a) { EIGSOL_EXACT return a.hi < 0.0 ? dd_neg(a) : a; }
EIGSOL_HD double dd_to_d(dd a) { return a.hi + a.lo; }   // = hi for a normalised value
EIGSOL_HD bool dd_le(dd a, dd b) { EIGSOL_EXACT return a.hi < b.hi || (a.hi == b.hi && a.lo <= b.lo); }

// ---- complex double-double: the arithmetic g++ emits for std::complex<long double>, in dd
EIGSOL_HD cdd cdd_from(dd re, dd im) { EIGSOL_EXACT return cdd{re, im}; }
EIGSOL_HD cdd cdd_add(cdd a, cdd b) { EIGSOL_EXACT return cdd{dd_add(a.re, b.re), dd_add(a.im, b.im)}; }
EIGSOL_HD cdd cdd_sub(cdd a, cdd b) { EIGSOL_EXACT return cdd{dd_sub(a.re, b.re), dd_sub(a.im, b.im)}; }
EIGSOL_HD cdd cdd_neg(cdd a) { EIGSOL_EXACT return cdd{dd_neg(a.re), dd_neg(a.im)}; }
EIGSOL_HD cdd cdd_conj(cdd a) { EIGSOL_EXACT return cdd{a.re, dd_neg(a.im)}; }
EIGSOL_HD cdd cdd_mul(cdd a, cdd b) {
    EIGSOL_EXACT
    return cdd{dd_sub(dd_mul(a.re, b.re), dd_mul(a.im, b.im)), dd_add(dd_mul(a.re, b.im), dd_mul(a.im, b.re))};
}
EIGSOL_HD cdd cdd_mul_r(cdd a, dd r) { EIGSOL_EXACT return cdd{dd_mul(a.re, r), dd_mul(a.im, r)}; }
EIGSOL_HD cdd cdd_div_r(cdd a, dd r) { EIGSOL_EXACT return cdd{dd_div(a.re, r), dd_div(a.im, r)}; }
EIGSOL_HD dd cdd_abs2(cdd a) { EIGSOL_EXACT return dd_add(dd_mul(a.re, a.re), dd_mul(a.im, a.im)); }
// exact scaling by 2^e (both parts; exact while lo stays a normal number)
EIGSOL_HD dd dd_ldexp(dd a, int e) { EIGSOL_EXACT return dd{std::ldexp(a.hi, e), std::ldexp(a.lo, e)}; }
EIGSOL_HD cdd cdd_ldexp(cdd a, int e) { EIGSOL_EXACT return cdd{dd_ldexp(a.re, e), dd_ldexp(a.im, e)}; }
// exponent that brings max(|re|, |im|) to [1, 2); 0 for zero or non-finite values (left unscaled)
EIGSOL_HD int cdd_scale_exp(cdd a) {
    const double m = std::fmax(std::fabs(a.re.hi), std::fabs(a.im.hi));
    return (m > 0.0 && m <= 1.7976931348623157e308) ? std::ilogb(m) : 0;
}
// |z| without forming |z|^2 at the input's scale: hypot-style, so |z| near 1e+-170 neither
// overflows nor underflows (the x87 long double it stands for has a far wider exponent range)
EIGSOL_HD dd cdd_abs(cdd a) {
    EIGSOL_EXACT
    const int e = cdd_scale_exp(a);
    return dd_ldexp(dd_sqrt(cdd_abs2(cdd_ldexp(a, -e))), e);
}
// a / b = a conj(b') / |b'|^2 * 2^-e with b' = b 2^-e of modulus ~1 (scaled division)
EIGSOL_HD cdd cdd_div(cdd a, cdd b) {
    EIGSOL_EXACT
    const int e = cdd_scale_exp(b);
    const cdd bs = cdd_ldexp(b, -e);
    const dd d = cdd_abs2(bs);
    return cdd_ldexp(cdd_div_r(cdd_mul(a, cdd_conj(bs)), d), -e);
}
EIGSOL_HD bool cdd_is_zero(cdd a) { EIGSOL_EXACT return a.re.hi == 0.0 && a.im.hi == 0.0; }

// ---- one interface over the two scalar types (kernels and host loops are templated on T)
template <class T> struct wide_ops;
template <> struct wide_ops<dd> {
    static constexpr bool complex = false;
    EIGSOL_HD static dd zero() { EIGSOL_EXACT return dd{0.0, 0.0}; }
    EIGSOL_HD static dd one() { EIGSOL_EXACT return dd{1.0, 0.0}; }
    EIGSOL_HD static dd add(dd a, dd b) { EIGSOL_EXACT return dd_add(a, b); }
    EIGSOL_HD static dd sub(dd a, dd b) { EIGSOL_EXACT return dd_sub(a, b); }
    EIGSOL_HD static dd mul(dd a, dd b) { EIGSOL_EXACT return dd_mul(a, b); }
    EIGSOL_HD static dd div(dd a, dd b) { EIGSOL_EXACT return dd_div(a, b); }
    EIGSOL_HD static dd mul_r(dd a, dd r) { EIGSOL_EXACT return dd_mul(a, r); }
    EIGSOL_HD static dd div_r(dd a, dd r) { EIGSOL_EXACT return dd_div(a, r); }
    EIGSOL_HD static dd conj(dd a) { EIGSOL_EXACT return a; }
    EIGSOL_HD static dd abs2(dd a) { EIGSOL_EXACT return dd_mul(a, a); }
    EIGSOL_HD static dd abs(dd a) { EIGSOL_EXACT return dd_abs(a); }
    EIGSOL_HD static bool is_zero(dd a) { EIGSOL_EXACT return dd_is_zero(a); }
    EIGSOL_HD static dd from_re(dd r) { EIGSOL_EXACT return r; }
    EIGSOL_HD static dd real(dd a) { EIGSOL_EXACT return a; }
    EIGSOL_HD static dd imag(dd) { EIGSOL_EXACT return dd{0.0, 0.0}; }
    EIGSOL_HD static dd make(dd re, dd) { EIGSOL_EXACT return re; }
    EIGSOL_HD static double hi(dd a) { EIGSOL_EXACT return a.hi; }
    EIGSOL_HD static dd ldexp(dd a, int e) { EIGSOL_EXACT return dd_ldexp(a, e); }
    EIGSOL_HD static double maxabs(dd a) { return std::fabs(a.hi); }
};
template <> struct wide_ops<cdd> {
    static constexpr bool complex = true;
    EIGSOL_HD static cdd zero() { EIGSOL_EXACT return cdd{{0.0, 0.0}, {0.0, 0.0}}; }
    EIGSOL_HD static cdd one() { EIGSOL_EXACT return cdd{{1.0, 0.0}, {0.0, 0.0}}; }
    EIGSOL_HD static cdd add(cdd a, cdd b) { EIGSOL_EXACT return cdd_add(a, b); }
    EIGSOL_HD static cdd sub(cdd a, cdd b) { EIGSOL_EXACT return cdd_sub(a, b); }
    EIGSOL_HD static cdd mul(cdd a, cdd b) { EIGSOL_EXACT return cdd_mul(a, b); }
    EIGSOL_HD static cdd div(cdd a, cdd b) { EIGSOL_EXACT return cdd_div(a, b); }
    EIGSOL_HD static cdd mul_r(cdd a, dd r) { EIGSOL_EXACT return cdd_mul_r(a, r); }
    EIGSOL_HD static cdd div_r(cdd a, dd r) { EIGSOL_EXACT return cdd_div_r(a, r); }
    EIGSOL_HD static cdd conj(cdd a) { EIGSOL_EXACT return cdd_conj(a); }
    EIGSOL_HD static dd abs2(cdd a) { EIGSOL_EXACT return cdd_abs2(a); }
    EIGSOL_HD static dd abs(cdd a) { EIGSOL_EXACT return cdd_abs(a); }
    EIGSOL_HD static bool is_zero(cdd a) { EIGSOL_EXACT return cdd_is_zero(a); }
    EIGSOL_HD static cdd from_re(dd r) { EIGSOL_EXACT return cdd{r, dd{0.0, 0.0}}; }
    EIGSOL_HD static dd real(cdd a) { EIGSOL_EXACT return a.re; }
    EIGSOL_HD static dd imag(cdd a) { EIGSOL_EXACT return a.im; }
    EIGSOL_HD static cdd make(dd re, dd im) { EIGSOL_EXACT return cdd{re, im}; }
    EIGSOL_HD static double hi(cdd a) { EIGSOL_EXACT return a.re.hi; }
    EIGSOL_HD static cdd ldexp(cdd a, int e) { EIGSOL_EXACT return cdd_ldexp(a, e); }
    EIGSOL_HD static double maxabs(cdd a) { return std::fmax(std::fabs(a.re.hi), std::fabs(a.im.hi)); }
};

}  // namespace eigsol
