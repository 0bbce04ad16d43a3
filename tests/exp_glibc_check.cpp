// exp_glibc_check.cpp -- CPU test driver (tests/test_exp_glibc.py): ggp::exp_glibc (ggp_prop.h,
// compiled for the host from the device source) against this process's libm exp(), bitwise.
//
//   exp_glibc_check N SEED   prints "<checked> <mismatches> <first mismatching x as hex or ->"
//
// Ranges: uniform in [-745, 710] (both special branches, the subnormal results), [-512, 512]
// (the main path), [-30, 30] (the propagator's arguments), |x| < 2^-50 (the tiny branch), every
// exponent's boundaries, and the specials (+-0, +-inf, NaN, the overflow/underflow edges).
#define GGP_HOST_SIM
#include "ggp_prop.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>


double (*ggp_hs_dawson)(double) = nullptr;
static double glibc_exp(double x) { return ::exp(x); }
namespace ggp {
double (*ggp_hs_exp)(double) = glibc_exp;
int ggp_hs_pow_libm = 0;
}

static uint64_t bits(double d)
{
    uint64_t u;
    memcpy(&u, &d, 8);
    return u;
}

int main(int argc, char **argv)
{
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    std::mt19937_64 rng(argc > 2 ? atol(argv[2]) : 1);
    long checked = 0, bad = 0;
    double first = 0.0;
    auto check = [&](double x) {
        volatile double xv = x;   // the libm call, not a folded constant
        const double a = ::exp(xv), b = ggp::exp_glibc(x, ggp_exp_tab);
        ++checked;
        const bool same = bits(a) == bits(b) || (std::isnan(a) && std::isnan(b));
        if (!same && bad++ == 0) first = x;
    };
    std::uniform_real_distribution<double> wide(-745.5, 710.0), main_(-512.0, 512.0), prop(-30.0, 30.0),
        tiny(-0x1p-50, 0x1p-50);
    for (long i = 0; i < n; ++i) {
        check(wide(rng));
        check(main_(rng));
        check(prop(rng));
        check(tiny(rng));
    }
    const double edges[] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 0x1p-54, -0x1p-54, 0x1.fffffffffffffp-55, 512.0,
                            -512.0, 0x1.fffffffffffffp8, 709.782712893384, 709.7827128933841, 1024.0, -1024.0,
                            -708.3964185322641, -745.1332191019411, -745.1332191019412, 1e300, -1e300,
                            0x1.62e42fefa39efp+9, -0x1.74910d52d3051p+9};
    for (const double e : edges)
        for (int k = -3; k <= 3; ++k) {
            double x = e;
            for (int j = 0; j < (k < 0 ? -k : k); ++j) x = std::nextafter(x, k < 0 ? -INFINITY : INFINITY);
            check(x);
        }
    if (bad) printf("%ld %ld %a\n", checked, bad, first);
    else printf("%ld 0 -\n", checked);
    return 0;
}
