/* ggp_oracle_sens.c -- TEST INFRASTRUCTURE ONLY.  Linked into oracle/liboracle_sens.so (the
 * oracle built with -DORA_EXPERIMENT), never into liboracle.so, the product or the bench.
 *
 * The conditioning probe of the parity tests: ora_set_exp_ulp_noise(seed) replaces exp() on
 * the propagator path (mean_cov_model.h tauint / mean_* / cov_*) by exp() moved one ulp up or
 * down at random -- the size of the ocml-vs-glibc difference the device sees.  An output that
 * moves under this noise by more than the parity tolerance is ill-conditioned in the
 * reference algorithm itself, and no device/CPU comparison of it is meaningful. */
#include <math.h>
#include <stdint.h>

#include "ggp_oracle.h"

static uint64_t g_state = 0;

static double exp_ulp_noise(double v)
{
    g_state ^= g_state << 13;
    g_state ^= g_state >> 7;
    g_state ^= g_state << 17;
    const double r = exp(v);
    return (g_state & 1) ? nextafter(r, INFINITY) : nextafter(r, -INFINITY);
}

/* seed 0: the unperturbed oracle */
void ora_set_exp_ulp_noise(uint64_t seed)
{
    g_state = seed ? seed : 0;
    ora_exp_hook = seed ? exp_ulp_noise : exp;
}

/* replace mean_cov_model by an external propagator (tools/hostsim.cpp: the device algorithm
 * compiled for the host), to measure what a reformulation of it does to the total */
void ora_set_mcm_hook(void (*fn)(double *, double *, double, const double *))
{
    ora_mcm_hook = fn;
}
