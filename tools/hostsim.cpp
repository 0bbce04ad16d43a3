// hostsim.cpp -- diagnostic only (never shipped): the device propagator compiled for the host
// (GGP_HOST_SIM: same source, glibc libm), exported for numerical experiments against the
// oracle (oracle/liboracle_sens.so ora_set_mcm_hook).  Build:
//   g++ -O2 -std=c++17 -ffp-contract=off -fPIC -shared -I gfp_gaussian_process_amd/csrc \
//       -o tools/libhostsim.so tools/hostsim.cpp
#define GGP_HOST_SIM
#include "ggp_outtab.h"
#include <cstring>

// the diagnostic hooks of the device headers (GGP_HOST_SIM): glibc's exp, the table Dawson
double (*ggp_hs_dawson)(double) = nullptr;
static double glibc_exp(double x) { return ::exp(x); }
namespace ggp {
double (*ggp_hs_exp)(double) = glibc_exp;
int ggp_hs_pow_libm = 0;
}

extern "C" {
// mean_cov_model through the lane schedule's expressions (ggp::propagate_lane)
void hs_mcm_lane(double *m, double *C, double t, const double *p)
{
    const ggp::OU P = ggp::make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    ggp::propagate_lane(m, C, t, P, ggp_dawson_coef);
}
// the same with the wave schedule's table-driven outputs (ggp_outtab.h)
void hs_mcm_tab(double *m, double *C, double t, const double *p)
{
    const ggp::OU P = ggp::make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    ggp::propagate_tab(m, C, t, P, ggp_dawson_coef);
}
}

extern "C" {
// both output forms on one (m, C): out_lane/out_tab = m[4] then C[16]
void hs_compare(const double *m, const double *C, double t, const double *p, double *out_lane, double *out_tab)
{
    for (int k = 0; k < 4; ++k) out_lane[k] = out_tab[k] = m[k];
    for (int k = 0; k < 16; ++k) out_lane[4 + k] = out_tab[4 + k] = C[k];
    hs_mcm_lane(out_lane, out_lane + 4, t, p);
    hs_mcm_tab(out_tab, out_tab + 4, t, p);
}
}

extern "C" {
// per-term values of the table form at (m, C): terms[64 * kOutL]
void hs_terms(const double *m, const double *C, double t, const double *p, double *terms)
{
    using namespace ggp;
    const OU P = make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    Step S;
    step_init(S, m, C, t, P);
    double X[NX];
    lane_exps(S, X, ggp::host_prop_tab(), std::make_index_sequence<NXT>{});
    X[X_ONE] = 1.0;
    double Dw[ND];
    lane_dawsons(S, Dw, ggp_dawson_coef, std::make_index_sequence<ND>{});
    double PW[NPW];
    for (int q = 0; q < 3; ++q) { PW[q] = pow_task(S, q); PW[3 + q] = 1.0 / PW[q]; }
    double I[NI];
    lane_taus(S, X, Dw, PW, I, std::make_index_sequence<NI>{});
    double V[V_N] = {1.0, S.bx, S.bg, S.bl - S.ml, S.bq - S.mq, S.Cxx, S.Cxg, S.Cxl, S.Cxq, S.Cgg, S.Cgl, S.Cgq, S.Cll,
                     S.Clq, S.Cqq, S.t};
    double Bv[BV_N];
    Bv[BV_ONE] = 1.0;
    for (int j = 0; j < NI; ++j) Bv[BV_I + j] = I[j];
    for (int j = 0; j < kNDerived; ++j) Bv[BV_R_EBT + j] = derived_basis(j, X, P.gl, S.t);
    for (int l = 0; l < 64; ++l)
        for (int q = 0; q < kOutL; ++q) {
            const OutTerm T = kOutTerm[l][q];
            terms[l * kOutL + q] = (((out_kappa(P, T.kap) * V[T.v1]) * V[T.v2]) * V[T.v3]) * Bv[T.basis];
        }
}
}

extern "C" {
// derived_generic (device form) against derived_basis (reference order): number of mismatching bits
int hs_check_derived(void)
{
    using namespace ggp;
    int bad = 0;
    for (int trial = 0; trial < 1000; ++trial) {
        double X[NX];
        for (int k = 0; k < NX; ++k) X[k] = exp(-0.001 * (trial % 97) - 0.01 * k);
        const double gl = 0.01 + 1e-4 * trial, t = 0.5 + 0.01 * (trial % 13);
        for (int j = 0; j < kNDerived; ++j) {
            const double a = derived_basis(j, X, gl, t), b = derived_generic(kDerived[j], X, gl, t);
            if (memcmp(&a, &b, 8)) ++bad;
        }
    }
    return bad;
}
}

// ---- the wave step (ggp_wave.h): 46 computed exponentials + 22 products,
// unified exp / Dawson Horner, monomial outputs -- propagation only (the oracle updates) ----
#include "ggp_wave.h"
#include <memory>

extern "C" {
void hs_mcm_wave(double *m, double *C, double t, const double *p)
{
    using namespace ggp;
    static std::unique_ptr<wave::HostWave> W;
    static double pc[11] = {0};
    if (!W || memcmp(pc, p, sizeof(pc))) {
        W.reset(new wave::HostWave(p));
        memcpy(pc, p, sizeof(pc));
    }
    double *lds = W->lds;
    for (int k = 0; k < 4; ++k) lds[wave::L_POST + k] = m[k];
    for (int k = 0; k < 16; ++k) lds[wave::L_POST + 4 + k] = C[k];
    double *V = lds + wave::L_V;
    const double v[14] = {m[0], m[1], m[2] - W->P.ml, m[3] - W->P.mq, C[0], C[1], C[2], C[3], C[5], C[6], C[7], C[10], C[11], C[15]};
    for (int k = 0; k < 14; ++k) V[1 + k] = v[k];
    W->propagate(t);
    double o[kOutN];
    out_finish([&](int k) { return lds[wave::L_OUT + k]; }, o);
    out_store(o, m, C);
}
}

// ---- the lane step with a chosen subset of the 22 product exponentials (kXP): products whose
// bit is clear in hs_xp_mask are computed directly (exp of their own argument) ----
static unsigned long long hs_xp_mask = ~0ull;
extern "C" {
void hs_set_xp_mask(unsigned long long m) { hs_xp_mask = m; }
void hs_mcm_lane_mask(double *m, double *C, double t, const double *p)
{
    using namespace ggp;
    const OU P = make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    Step S;
    step_init(S, m, C, t, P);
    double Xc[NXC], X[NXE];
    lane_exps_c(S, Xc, ggp::host_prop_tab(), std::make_index_sequence<NXC>{});
    lane_expand(Xc, X);
    for (int q = 0; q < NXP; ++q)
        if (!((hs_xp_mask >> q) & 1)) X[kXP[q].j] = exp_body(S, kXT[kXP[q].j], ggp::host_prop_tab());
    double Dw[ND];
    lane_dawsons(S, Dw, ggp_dawson_coef, std::make_index_sequence<ND>{});
    double PW[NPW];
    for (int q = 0; q < 3; ++q) { PW[q] = pow_task(S, q); PW[3 + q] = frcp(PW[q]); }
    double I[NI];
    lane_taus(S, X, Dw, PW, I, std::make_index_sequence<NI>{});
    outputs(S, I, X, m, C);
}
}
