// parity_attrib.cpp -- diagnostic only (never shipped, never loaded by tests or the bench).
//
// The lane schedule's total log-likelihood emulated on the host from the device source
// (GGP_HOST_SIM: ggp_prop.h / ggp_device.h compiled for x86-64), with each of the device's
// departures from the oracle's arithmetic behind a switch, so that tools/parity_attrib.py can
// switch them on one at a time on the example and attribute the GPU-vs-oracle gap:
//
//   contraction   per-expression fma (clang's fp contract(on)) -- a compile-time switch: the
//                 tool builds this file twice, with and without -DGGP_HOST_CONTRACT -mfma
//   exp           glibc's exp (the oracle's) or exp_ocml (ocml's sequence, the device's value)
//   products      the 22 product exponentials (kXP) on/off, one bit each
//   pow           tauint denominators as a^k sqrt(a) (device) or pow(a, k + 1/2) (oracle)
//   dawson        the table (device and oracle) or any other Dawson (e.g. the reference's
//                 Faddeeva::Dawson from oracle/_ref, passed as a function pointer)
//
// The traversal and cell body are loglik_lane_cell's (ggp_engine.hip): DFS pre-order over the
// roots, each cell from its parent's final state, one partial sum per cell added in DFS order.
//
// Build (tools/parity_attrib.py does this):
//   clang++ -O2 -std=c++17 -fPIC -shared -ffp-contract=off [-DGGP_HOST_CONTRACT -mfma]
//           -I gfp_gaussian_process_amd/csrc -I oracle -o /tmp/libpa.so tools/parity_attrib.cpp
#define GGP_HOST_SIM
#include "ggp_prop.h"
#include "ggp_oracle.h"

#include <cmath>
#include <cstring>
#include <vector>

double (*ggp_hs_dawson)(double) = nullptr;
static double glibc_exp(double x) { return ::exp(x); }
namespace ggp {
double (*ggp_hs_exp)(double) = glibc_exp;
int ggp_hs_pow_libm = 0;
}

static double exp_ocml_host(double x) { return ggp::exp_ocml(x); }
static unsigned long long g_xp_mask = ~0ull;

namespace {
using namespace ggp;

// propagate_lane with the products whose bit is clear in g_xp_mask formed directly
void propagate_masked(double *m, double *C, const double t, const OU &P)
{
    Step S;
    step_init(S, m, C, t, P);
    double Xc[NXC], X[NXE];
    lane_exps_c(S, Xc, host_prop_tab(), std::make_index_sequence<NXC>{});
    lane_expand(Xc, X);
    for (int q = 0; q < NXP; ++q)
        if (!((g_xp_mask >> q) & 1)) X[kXP[q].j] = exp_body(S, kXT[kXP[q].j], host_prop_tab());
    double Dw[ND];
    lane_dawsons(S, Dw, host_prop_tab(), std::make_index_sequence<ND>{});
    double PW[NPW];
    for (int q = 0; q < 3; ++q) {
        PW[q] = pow_task(S, q);
        PW[3 + q] = frcp(PW[q]);
    }
    double I[NI];
    lane_taus(S, X, Dw, PW, I, std::make_index_sequence<NI>{});
    outputs(S, I, X, m, C);
}

std::vector<int64_t> dfs_preorder(const ora_forest *f)
{
    std::vector<int64_t> order, stack;
    for (int64_t r = 0; r < f->n_cells; ++r) {
        if (f->parent[r] != -1) continue;
        stack.push_back(r);
        while (!stack.empty()) {
            const int64_t c = stack.back();
            stack.pop_back();
            order.push_back(c);
            if (f->d2[c] >= 0) stack.push_back(f->d2[c]);
            if (f->d1[c] >= 0) stack.push_back(f->d1[c]);
        }
    }
    return order;
}
}  // namespace

extern "C" {
// exp_kind: 0 glibc, 1 exp_ocml; xp_mask: bit q set = product q of kXP; pow_libm: 1 = pow();
// dawson: nullptr = the table, else every Dawson value from it
void pa_configure(int exp_kind, unsigned long long xp_mask, int pow_libm, double (*dawson)(double))
{
    ggp::ggp_hs_exp = exp_kind ? exp_ocml_host : glibc_exp;
    g_xp_mask = xp_mask;
    ggp::ggp_hs_pow_libm = pow_libm;
    ggp_hs_dawson = dawson;
}

int pa_contracted(void)
{
#ifdef GGP_HOST_CONTRACT
    return 1;
#else
    return 0;
#endif
}

// one evaluation (the 2-arg total_likelihood) on the carried state [n_cells x 20]
double pa_total(const ora_forest *f, const double *p, double *state)
{
    const OU ou = make_ou(p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
    const double two_log_2pi = 2 * log(2 * M_PI), log2 = log(2.);
    double total = 0.0;
    for (const int64_t c : dfs_preorder(f)) {
        double m[4], C[16];
        const int64_t r0 = f->row_off[c], r1 = f->row_off[c + 1];
        double dt = 0.0;
        bool pending = false;
        const int par = f->parent[c];
        if (par < 0) {   // cell_prologue / root_init
            memcpy(C, state + 20 * c + 4, sizeof C);
            m[0] = f->root_mean_xg[0];
            m[1] = f->root_mean_xg[1];
            C[0] = f->root_var_xg[0];
            C[5] = f->root_var_xg[1];
            m[2] = p[0];
            m[3] = p[3];
            C[10] = p[2] / (2. * p[1]);
            C[15] = p[5] / (2. * p[4]);
        } else {
            memcpy(m, state + 20 * par, sizeof m);
            memcpy(C, state + 20 * par + 4, sizeof C);
            dt = f->time[r0] - f->time[f->row_off[par + 1] - 1];
            pending = true;
        }
        bool divide = pending;
        double cl = 0.0;
        double t_cur = f->time[r0];
        for (int64_t r = r0; r < r1; ++r) {
            const double t_next = r + 1 < r1 ? f->time[r + 1] : 0.0;
            if (pending) {
                propagate_masked(m, C, dt, ou);
                if (divide) {
                    division_map(m, C, p[9], p[10], f->div_binomial, log2);
                    divide = false;
                }
            }
            const double x0 = f->log_length[r] - m[0], x1 = f->fp[r] - m[1];
            ggp_innov v;
            ggp_innovation(m, C, p[7], p[8], f->noise_scaled, f->fp_auto, v);
            cl += ggp_ll_term(x0, x1, v, two_log_2pi);
            ggp_posterior(m, C, x0, x1, v);
            pending = r + 1 < r1;
            if (pending) dt = t_next - t_cur;
            t_cur = t_next;
        }
        memcpy(state + 20 * c, m, sizeof m);
        memcpy(state + 20 * c + 4, C, sizeof C);
        total += cl;
    }
    return total;
}
}
