// CPU check of the Nelder-Mead lookahead (ggp_nelder_mead.h): a stateful objective serves calls
// from the speculated tree while they match; the run must make the same calls with the same
// values as without the lookahead, and (on these smooth test functions) every call after the
// first must be served from a tree.  Prints "same <calls> <served> <launches> <max nodes>".
#include "ggp_nelder_mead.h"
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char **argv)
{
    const int n = argc > 1 ? std::atoi(argv[1]) : 10;
    const int fixed = argc > 2 ? std::atoi(argv[2]) : -1;   // one dimension with lb == ub
    auto obj = [&](const double *x) {
        double s = 0;
        for (int i = 0; i < n; ++i) {
            const double d = x[i] - 0.3 * (i + 1);
            s += (1 + i) * d * d + 0.1 * std::sin(3 * x[i]);
        }
        return s;
    };
    std::vector<double> lb(n, -5), ub(n, 5), dx(n, 0.5), x0(n, 0.0);
    if (fixed >= 0) lb[fixed] = ub[fixed] = 0.0;
    std::vector<std::vector<double>> calls_plain, calls_look;
    auto run = [&](bool look_on, std::vector<std::vector<double>> &calls, long &served, long &launches, size_t &max_nodes) {
        std::vector<std::vector<double>> nodes;
        std::vector<int> pred;
        int cur = -1;
        bool active = false;
        auto find = [&](const double *x) {
            if (!active) return -1;
            for (size_t k = 0; k < nodes.size(); ++k)
                if (pred[k] == cur && std::memcmp(nodes[k].data(), x, sizeof(double) * n) == 0) return (int)k;
            return -1;
        };
        ggp_nm::Lookahead look;
        look.need = [&](const double *x) { return find(x) < 0; };
        look.tree = [&](const std::vector<std::vector<double>> &xs, const std::vector<int> &p) {
            for (size_t k = 0; k < xs.size(); ++k)
                if (p[k] >= (int)k || p[k] < -1) std::abort();   // parents come first
            nodes = xs;
            pred = p;
            cur = -1;
            active = true;
            ++launches;
            if (xs.size() > max_nodes) max_nodes = xs.size();
        };
        ggp_nm::Objective f = [&](const double *x, double *v) {
            calls.emplace_back(x, x + n);
            const int k = find(x);
            if (k >= 0) {
                cur = k;
                ++served;
            } else {
                active = false;
            }
            *v = obj(x);
            return true;
        };
        std::vector<double> x(x0);
        double minf = 0;
        ggp_nm::Stats st;
        ggp_nm::minimize(n, f, lb.data(), ub.data(), x.data(), dx.data(), 1e-8, 0, &minf, st, look_on ? &look : nullptr);
        return minf;
    };
    long s0 = 0, l0 = 0, s1 = 0, l1 = 0;
    size_t m0 = 0, m1 = 0;
    const double a = run(false, calls_plain, s0, l0, m0), b = run(true, calls_look, s1, l1, m1);
    const bool same = a == b && calls_plain == calls_look;
    std::printf("%s %zu %ld %ld %zu\n", same ? "same" : "differ", calls_look.size(), s1, l1, m1);
    return 0;
}
