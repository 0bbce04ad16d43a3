// ggp_cli.cpp -- the command-line surface of the reference (src/main.cpp) over the MI355X
// engine: same flags, defaults, checks, output files and formats; the likelihood and the
// smoother run on the GPU through include/ggp.h, ingest through include/ggp_host.h.
//
//   -m  run_minimization      main.cpp:23-77    (minimize_wrapper[_log_params], error bars,
//                                                final csv, generated parameter file)
//   -s  run_bound_1dscan      main.cpp:80-114
//   -p  run_prediction_segments main.cpp:117-146 (write_predictions_to_file)
//   -e  additive: one total log-likelihood at the parameter files' values
//   -hb additive: -m's error bars from one batched call (ggp_total_loglik_batch)
//   -j  run_joint_distribution  main.cpp:150-186 (collect_joint_distributions' dense joint
//                                matrix, correlation_tree.h:9-23, 96-126, 588-648, 786-791);
//                                as in the reference, -j implies -p (main.cpp:265-268)
//
// Output text is produced with the same iostream manipulators as the reference, so the files
// are byte-identical given identical numbers.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <map>
#include <numeric>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ggp.h"
#include "ggp_host.h"
#include "ggp_nelder_mead.h"
#include "ggp_text.h"

namespace {

std::ofstream g_log;        // _file_log
std::ofstream g_iter;       // _file_iteration
int g_iteration = 0;        // _iteration
int g_print_level = 0;      // _print_level
bool g_save_ll = false;     // _save_ll

// GGP_TIMING=1 (additive, diagnostic): wall seconds of the phases to stderr; the log files keep
// the reference's content
struct PhaseClock {
    const bool on = std::getenv("GGP_TIMING") && std::getenv("GGP_TIMING")[0] == '1';
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void mark(const char *what)
    {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ggp timing] %-28s %9.3f s\n", what, std::chrono::duration<double>(t - t0).count());
        t0 = t;
    }
};
PhaseClock g_clock;

// ---- utils.h ------------------------------------------------------------------------------
std::vector<std::string> split_string_at(std::string s, const std::string &delimiter = ",")
{
    std::vector<std::string> out;
    size_t pos;
    while ((pos = s.find(delimiter)) != std::string::npos) {
        out.push_back(s.substr(0, pos));
        s.erase(0, pos + delimiter.length());
    }
    out.push_back(s);
    return out;
}

std::string trim(const std::string &str, char trim_char = ' ')
{
    const size_t first = str.find_first_not_of(trim_char);
    if (first == std::string::npos) return str;
    const size_t last = str.find_last_not_of(' ');
    return str.substr(first, last - first + 1);
}

std::string pad_str(std::string s, size_t num)
{
    if (num > s.size()) s.insert(s.end(), num - s.size(), ' ');
    return s;
}

std::string pad_str(double d, size_t num)
{
    std::stringstream b;
    b << d;
    return pad_str(b.str(), num);
}

std::string file_base(const std::string &infile)
{
    const auto parts = split_string_at(infile, "/");
    const auto base = split_string_at(parts.back(), ".");
    std::string out;
    for (size_t i = 0; i + 1 < base.size(); ++i) {
        if (i > 0) out += '.';
        out += base[i];
    }
    return out;
}

std::string default_out_dir(const std::string &infile)
{
    const auto parts = split_string_at(infile, "/");
    const auto base = split_string_at(parts.back(), ".");
    std::string out;
    for (size_t i = 0; i + 1 < parts.size(); ++i) out += parts[i] + "/";
    for (size_t i = 0; i + 1 < base.size(); ++i) {
        if (i > 0) out += '.';
        out += base[i];
    }
    return out + "_out/";
}

std::string out_dir(std::map<std::string, std::string> &args)
{
    std::string d;
    if (!args.count("outdir")) {
        d = default_out_dir(args["infile"]);
    } else {
        d = args["outdir"];
        if (d.back() != '/') d += "/";
    }
    std::filesystem::create_directory(d);
    return d;
}

std::string add_segment_to_filename(const std::string &name, int segment)
{
    return segment == -1 ? name : name + "_segment" + std::to_string(segment);
}

template <typename T>
std::vector<T> arange(T start, T stop, T step)
{
    std::vector<T> v;
    for (T x = start; x < stop; x += step) v.push_back(x);
    return v;
}

// ---- Parameters.h -------------------------------------------------------------------------
struct Params {
    ggp_param_set p{};
    double final_[GGP_N_PARAMS] = {};
    bool minimized[GGP_N_PARAMS] = {};
    bool fixed(int i) const { return p.kind[i] == 0; }
    bool free_(int i) const { return p.kind[i] == 1; }
    bool bound(int i) const { return p.kind[i] == 2; }
    std::string name(int i) const { return p.name[i]; }
    bool has_nonfixed() const
    {
        for (int i = 0; i < GGP_N_PARAMS; ++i)
            if (!fixed(i)) return true;
        return false;
    }
    std::vector<double> get_final() const
    {
        std::vector<double> v(GGP_N_PARAMS);
        for (int i = 0; i < GGP_N_PARAMS; ++i) v[i] = minimized[i] ? final_[i] : p.init[i];
        return v;
    }
    void set_final(const std::vector<double> &v)
    {
        for (int i = 0; i < GGP_N_PARAMS; ++i) {
            final_[i] = v[i];
            minimized[i] = true;
        }
    }
    std::vector<int> non_fixed() const
    {
        std::vector<int> idx;
        for (int i = 0; i < GGP_N_PARAMS; ++i)
            if (!fixed(i)) idx.push_back(i);
        return idx;
    }
    void to_csv(std::ostream &file) const   // Parameter_set::to_csv (Parameters.h:201-224)
    {
        file << "no,name,type,init,step,lower_bound,upper_bound,final\n";
        for (int i = 0; i < GGP_N_PARAMS; ++i) {
            file << i << ",";
            if (fixed(i)) {
                file << name(i) << "," << "fixed" << "," << p.init[i] << ", , , ,";
            } else if (bound(i)) {
                file << name(i) << "," << "bound" << "," << p.init[i] << "," << p.step[i] << "," << p.lower[i] << ","
                     << p.upper[i] << ",";
            } else {
                file << name(i) << "," << "free" << "," << p.init[i] << "," << p.step[i] << ", , ,";
            }
            if (minimized[i]) file << final_[i];
            file << "\n";
        }
    }
    void to_csv(const std::string &outfile, std::ios_base::openmode mode = std::ios_base::out) const
    {
        std::ofstream f(outfile, mode);
        to_csv(f);
    }
};

std::ostream &operator<<(std::ostream &os, const Params &P)   // Parameters.h:300-334
{
    const std::vector<int> w{4, 15, 8, 20, 20, 15, 15};
    os << pad_str("No", w[0]) << pad_str("Name", w[1]) << pad_str("Type", w[2]) << pad_str("Init", w[3])
       << pad_str("Step", w[4]) << pad_str("Bounds", w[5]) << "\n";
    for (int i = 0; i < std::accumulate(w.begin(), w.end(), 0); ++i) os << "_";
    os << "\n";
    for (int i = 0; i < GGP_N_PARAMS; ++i) {
        os << pad_str(std::to_string(i) + ":", w[0]);
        if (P.fixed(i)) {
            os << pad_str(P.name(i), w[1]) << pad_str("(fixed)", w[2]) << pad_str(P.p.init[i], w[3])
               << pad_str("", w[4] + w[5] + w[6]);
        } else if (P.bound(i)) {
            os << pad_str(P.name(i), w[1]) << pad_str("(bound)", w[2]) << pad_str(P.p.init[i], w[3])
               << pad_str(P.p.step[i], w[4]) << pad_str(P.p.lower[i], w[5]) << pad_str(P.p.upper[i], w[6]);
        } else {
            os << pad_str(P.name(i), w[1]) << pad_str("(free)", w[2]) << pad_str(P.p.init[i], w[3])
               << pad_str(P.p.step[i], w[4]) << pad_str("", w[5] + w[6]);
        }
        if (P.minimized[i] && !P.fixed(i)) os << " -> " << P.final_[i];
        os << "\n";
    }
    return os;
}

std::string outfile_param_code(const Params &P)   // predictions.h:505-520
{
    std::string code = "_f";
    for (int i = 0; i < GGP_N_PARAMS; ++i)
        if (!P.bound(i) && !P.fixed(i)) code += std::to_string(i);
    code += "_b";
    for (int i = 0; i < GGP_N_PARAMS; ++i)
        if (P.bound(i)) code += std::to_string(i);
    return code;
}

// ---- the objective on the GPU (likelihood.h:125-174) --------------------------------------
struct Objective {
    ggp_forest *forest = nullptr;
    ggp_host_forest *host = nullptr;
    const ggp_forest_desc *desc = nullptr;
    // -m lookahead (ggp_nm::Lookahead): a tree of the run's possible next calls (node k from the
    // state node pred[k] leaves; -1: the carried state), evaluated in one ggp_total_loglik_tree
    // call; total_likelihood serves a call from the children of the last node served
    struct Ahead {
        bool active = false, off = false;
        int n = 0, cur = -1;
        std::vector<double> pts, ll;
        std::vector<int32_t> pred, st;
        std::vector<int64_t> nc, nr;
    } ahead;
};

void log_iteration(const std::vector<double> &p, double tl, int iteration)
{
    g_iter << iteration << ",";
    for (double v : p) g_iter << std::setprecision(20) << v << ",";
    g_iter << std::setprecision(30) << tl << std::setprecision(15) << "\n";
}

// +ll; throws std::domain_error("Likelihood is Nan") after the reference's side effects
// what total_likelihood does after an evaluation (likelihood.h:71-93, 137-158): the NaN log and
// exception, the iteration count, the -m iteration log and the print-level line
double account(const std::vector<double> &params, Objective &o, int rc, double ll, int64_t nc, int64_t nr)
{
    if (rc == GGP_ENAN) {
        if (g_save_ll) log_iteration(params, ll, g_iteration + 1);
        g_log << "\n(sc_likelihood) ERROR: Log likelihood is Nan\n";
        g_log << "____________________________________________\n";
        if (nc >= 0) {
            const double t = o.desc->time[o.desc->row_offset[nc] + nr];
            g_log << "cell_id: " << ggp_host_forest_cell_id(o.host, nc) << ", at time " << t << "\n";
        }
        g_log << g_iteration + 1 << ": ";
        for (double v : params) g_log << v << ", ";
        g_log << "ll=" << std::setprecision(10) << ll << "\n";
        g_iter.close();
        throw std::domain_error("Likelihood is Nan");
    }
    if (rc != GGP_OK) throw std::runtime_error(std::string("GPU likelihood failed: ") + ggp_strerror(rc));
    ++g_iteration;
    if (g_save_ll) log_iteration(params, ll, g_iteration);
    if (g_print_level > 0) {
        std::cout << g_iteration << ": ";
        for (double v : params) std::cout << std::setprecision(20) << v << ", ";
        std::cout << "ll=" << std::setprecision(30) << ll << std::setprecision(15) << "\n";
    }
    return ll;
}

// evaluate a tree of calls ahead in one speculative launch; nothing changes until the calls come
void look_ahead(Objective &o, const std::vector<std::vector<double>> &pts, const std::vector<int> &pred)
{
    Objective::Ahead &a = o.ahead;
    a.active = false;
    if (a.off || pts.empty()) return;
    a.n = (int)pts.size();
    a.cur = -1;
    a.pts.resize((size_t)a.n * GGP_N_PARAMS);
    for (int k = 0; k < a.n; ++k) std::memcpy(&a.pts[(size_t)k * GGP_N_PARAMS], pts[k].data(), GGP_N_PARAMS * sizeof(double));
    a.pred.assign(pred.begin(), pred.end());
    a.ll.assign((size_t)a.n, 0.0);
    a.st.assign((size_t)a.n, 0);
    a.nc.assign((size_t)a.n, -1);
    a.nr.assign((size_t)a.n, -1);
    const int rc = ggp_total_loglik_tree(o.forest, a.n, a.pts.data(), a.pred.data(), a.ll.data(), a.st.data(),
                                         a.nc.data(), a.nr.data());
    if (rc == GGP_EINVAL) {   // no path launch on this handle (or too many points): no lookahead
        a.off = true;
        return;
    }
    if (rc != GGP_OK) throw std::runtime_error(std::string("GPU likelihood failed: ") + ggp_strerror(rc));
    a.active = true;
}

// the node that serves the call `params` next: a child of the last node served, else -1
int ahead_node(const Objective &o, const double *params)
{
    const Objective::Ahead &a = o.ahead;
    if (!a.active) return -1;
    for (int k = 0; k < a.n; ++k)
        if (a.pred[(size_t)k] == a.cur &&
            std::memcmp(params, &a.pts[(size_t)k * GGP_N_PARAMS], GGP_N_PARAMS * sizeof(double)) == 0)
            return k;
    return -1;
}

double total_likelihood(const std::vector<double> &params, Objective &o)
{
    Objective::Ahead &a = o.ahead;
    if (a.active) {
        int k = ahead_node(o, params.data());
        // a node whose speculative launch stalled (GGP_ETIMEOUT: the lookahead's schedule, not the
        // call) is not served: the call runs below from the carried state, the last node served
        if (k >= 0 && a.st[(size_t)k] == GGP_ETIMEOUT) k = -1;
        if (k >= 0) {   // evaluated ahead: its state becomes the carried state, its value the call's
            a.cur = k;
            const int rc = ggp_keep_point_state(o.forest, k);
            if (rc != GGP_OK) throw std::runtime_error(std::string("ggp_keep_point_state: ") + ggp_strerror(rc));
            return account(params, o, a.st[(size_t)k], a.ll[(size_t)k], a.nc[(size_t)k], a.nr[(size_t)k]);
        }
        a.active = false;   // not foreseen: the carried state is the last served node's
    }
    double ll = 0;
    int64_t nc = -1, nr = -1;
    const int rc = ggp_total_loglik(o.forest, params.data(), &ll, &nc, &nr);
    return account(params, o, rc, ll, nc, nr);
}

// a known sequence of total_likelihood calls (each from the state the previous left) as one
// ggp_total_loglik_chain call: the same values, log lines and exceptions, point by point
std::vector<double> total_likelihood_chain(const std::vector<double> &pts, Objective &o)
{
    const int32_t n = (int32_t)(pts.size() / GGP_N_PARAMS);
    o.ahead.active = false;
    std::vector<double> ll((size_t)n, 0.0);
    int32_t n_ok = 0;
    int64_t nc = -1, nr = -1;
    const int rc = ggp_total_loglik_chain(o.forest, n, pts.data(), ll.data(), &n_ok, &nc, &nr);
    auto point = [&](int32_t i) {
        return std::vector<double>(pts.begin() + (size_t)i * GGP_N_PARAMS, pts.begin() + (size_t)(i + 1) * GGP_N_PARAMS);
    };
    for (int32_t i = 0; i < n_ok; ++i) account(point(i), o, GGP_OK, ll[(size_t)i], -1, -1);
    if (rc != GGP_OK) {
        if (n_ok < n) account(point(n_ok), o, rc, ll[(size_t)n_ok], nc, nr);   // throws
        throw std::runtime_error(std::string("GPU likelihood failed: ") + ggp_strerror(rc));
    }
    return ll;
}

// -g / -chunk (additive): the devices the forest is sharded over (default: every
// visible device; repeats = logical shards on one device) and the rows per shard cap
std::vector<int32_t> g_devices;
int64_t g_max_shard_rows = 0;

struct Forest {
    ggp_host_forest *host = nullptr;
    ggp_forest_desc desc{};
    ggp_forest *gpu = nullptr;
    ~Forest()
    {
        if (gpu) ggp_forest_destroy(gpu);
        if (host) ggp_host_forest_free(host);
    }
};

void build_forest(Forest &F, const ggp_dataset *d, int segment, const std::string &noise, const std::string &div)
{
    if (ggp_forest_build(d, segment, noise == "scaled", div == "binomial", &F.host) != GGP_OK)
        throw std::invalid_argument(ggp_host_last_error());
    ggp_host_forest_desc(F.host, &F.desc);
    F.desc.n_devices = g_devices.empty() ? GGP_ALL_DEVICES : (int32_t)g_devices.size();
    F.desc.devices = g_devices.empty() ? nullptr : g_devices.data();
    F.desc.max_shard_rows = g_max_shard_rows;
    F.desc.kernel = GGP_KERNEL_AUTO;
    const int rc = ggp_forest_create(&F.desc, &F.gpu);
    if (rc != GGP_OK) throw std::runtime_error(std::string("ggp_forest_create: ") + ggp_strerror(rc));
}

// ---- -m (minimizer_nlopt.h, likelihood.h:211-350) ------------------------------------------
double minimize(Objective &o, Params &P, double tolerance, bool log_space)
{
    const int n = GGP_N_PARAMS;
    std::vector<double> lb(n), ub(n), step(n), x(n);
    for (int i = 0; i < n; ++i) {
        const double start = P.minimized[i] ? P.final_[i] : P.p.init[i];
        x[i] = log_space ? std::log(start) : start;
        if (P.fixed(i)) {
            step[i] = 1.;
            lb[i] = ub[i] = log_space ? std::log(P.p.init[i]) : P.p.init[i];
        } else {
            step[i] = log_space ? std::log(1. + P.p.step[i] / P.p.init[i]) : P.p.step[i];
            lb[i] = log_space ? std::log(P.p.lower[i]) : P.p.lower[i];
            ub[i] = log_space ? std::log(P.p.upper[i]) : P.p.upper[i];
        }
    }
    g_save_ll = true;
    g_log << "Optimization algorithm: Nelder-Mead simplex algorithm (local, no-derivative) Tolerance: " << tolerance
          << "\n";
    g_iteration = 0;
    std::vector<double> pv(n);
    const ggp_nm::Objective f = [&](const double *xx, double *v) {
        for (int i = 0; i < n; ++i) pv[i] = log_space ? std::exp(xx[i]) : xx[i];
        *v = -total_likelihood(pv, o);   // throws on NaN, unwinding the optimiser
        return true;
    };
    // the lookahead, in parameter space (log_space: the exponentials the objective takes)
    auto to_params = [&](const double *src) {
        std::vector<double> v((size_t)n);
        for (int i = 0; i < n; ++i) v[i] = log_space ? std::exp(src[i]) : src[i];
        return v;
    };
    ggp_nm::Lookahead look;
    look.need = [&](const double *xx) { return ahead_node(o, to_params(xx).data()) < 0; };
    look.tree = [&](const std::vector<std::vector<double>> &xs, const std::vector<int> &pred) {
        std::vector<std::vector<double>> ps;
        for (const auto &xx : xs) ps.push_back(to_params(xx.data()));
        look_ahead(o, ps, pred);
    };
    if (const char *e = std::getenv("GGP_NM_AHEAD_DEPTH")) look.depth = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("GGP_NM_AHEAD_NODES")) look.max_nodes = std::max(1, std::atoi(e));
    const char *lk = std::getenv("GGP_NM_LOOKAHEAD");
    const bool use_look = !(lk && std::atoi(lk) == 0);
    double minf = 0;
    ggp_nm::Stats st;
    ggp_nm::Result r;
    try {
        r = ggp_nm::minimize(n, f, lb.data(), ub.data(), x.data(), step.data(), tolerance, 0, &minf, st,
                             use_look ? &look : nullptr);
        o.ahead.active = false;
        if (g_clock.on)
            std::fprintf(stderr, "[ggp timing] -m: %ld calls, %ld iterations (%ld expansions, %ld accepts, %ld contractions, %ld shrinks)\n",
                         st.nevals, st.iterations, st.expansions, st.accepts, st.contractions, st.shrinks);
        g_clock.mark("-m: minimised");
    } catch (std::exception &e) {
        o.ahead.active = false;
        g_log << "(minimize_wrapper) ERROR: Log likelihood optimization failed (" << e.what() << ")" << std::endl;
        throw;
    }
    if (r == ggp_nm::INVALID_ARGS) throw std::invalid_argument("nlopt invalid argument");
    if (r == ggp_nm::FAILURE) throw std::runtime_error("nlopt failure");
    g_save_ll = false;
    g_log << "Found maximum: log likelihood = " << std::setprecision(20) << -minf << std::setprecision(10) << "\n";
    if (log_space)
        for (int i = 0; i < n; ++i) x[i] = std::exp(x[i]);
    P.set_final(x);
    g_log << P << std::endl;
    return -minf;
}

// -hb (additive, opt-in): num_hessian_ll's 4 k^2 points (likelihood.h:211-258, same order, steps
// and expression as ggp_num_hessian) in one ggp_total_loglik_batch call, each point from the
// carried state left by the optimiser instead of chained from point to point
// num_hessian_ll's points (likelihood.h:211-258): for i, j of the free parameters, x +- h_i e_i
// +- h_j e_j in the order ++, +-, -+, --, h = max(x epsilon, 1e-12) (the steps of ggp_num_hessian)
void hessian_points(const std::vector<double> &x, const std::vector<int> &idx, double epsilon, std::vector<double> &h,
                    std::vector<double> &pts)
{
    const int k = (int)idx.size();
    h.assign((size_t)k, 0.0);
    pts.clear();
    for (int a = 0; a < k; ++a) h[a] = std::max(x[idx[a]] * epsilon, 1e-12);
    for (int a = 0; a < k; ++a)
        for (int b = 0; b < k; ++b)
            for (int q = 0; q < 4; ++q) {
                std::vector<double> xx = x;
                const int ii = idx[a], jj = idx[b];
                xx[ii] = q < 2 ? xx[ii] + h[a] : xx[ii] - h[a];
                xx[jj] = q % 2 == 0 ? xx[jj] + h[b] : xx[jj] - h[b];
                pts.insert(pts.end(), xx.begin(), xx.end());
            }
}

void num_hessian_batched(Objective &o, const std::vector<double> &x, const std::vector<int> &idx, double epsilon,
                         std::vector<double> &H)
{
    const int k = (int)idx.size();
    std::vector<double> h, pts;
    hessian_points(x, idx, epsilon, h, pts);
    const int n = 4 * k * k;
    std::vector<double> ll(n);
    std::vector<int32_t> st(n);
    const int rc = ggp_total_loglik_batch(o.forest, n, pts.data(), ll.data(), st.data());
    if (rc != GGP_OK) throw std::runtime_error(std::string("GPU batched likelihood failed: ") + ggp_strerror(rc));
    for (int i = 0; i < n; ++i)
        if (st[i] == GGP_ENAN) {
            g_log << "\n(num_hessian_batched) ERROR: Log likelihood is Nan\n";
            throw std::domain_error("Likelihood is Nan");
        }
    g_iteration += n;
    for (int a = 0; a < k; ++a)
        for (int b = 0; b < k; ++b) {
            const double *l = &ll[(size_t)4 * (a * k + b)];
            H[(size_t)a * k + b] = (l[0] - l[1] - l[2] + l[3]) / (4 * h[a] * h[b]);
        }
}

bool g_batched_hessian = false;

std::vector<double> ll_error_bars(Params &P, Objective &o, double epsilon)
{
    const std::vector<double> x = P.get_final();
    const std::vector<int> idx = P.non_fixed();
    const int k = (int)idx.size();
    std::vector<double> H((size_t)k * k), Hi((size_t)k * k);
    if (g_batched_hessian) {
        num_hessian_batched(o, x, idx, epsilon, H);
        ggp_inverse_pplu(k, H.data(), Hi.data());
        std::vector<double> err;
        for (int i = 0; i < k; ++i) err.push_back(-Hi[(size_t)i * k + i]);
        return err;
    }
    // num_hessian_ll's 4 k^2 calls, chained through the carried state as the reference makes them,
    // in one ggp_total_loglik_chain call; H as ggp_num_hessian forms it
    std::vector<double> h((size_t)k), pts;
    hessian_points(x, idx, epsilon, h, pts);
    const std::vector<double> ll = total_likelihood_chain(pts, o);
    for (int a = 0; a < k; ++a)
        for (int b = 0; b < k; ++b) {
            const double *l = &ll[(size_t)4 * (a * k + b)];
            H[(size_t)a * k + b] = (l[0] - l[1] - l[2] + l[3]) / (4 * h[a] * h[b]);
        }
    ggp_inverse_pplu(k, H.data(), Hi.data());
    std::vector<double> err;
    for (int i = 0; i < k; ++i) err.push_back(-Hi[(size_t)i * k + i]);
    return err;
}

void run_minimization(Objective &o, Params &P, std::map<std::string, std::string> &args, int segment, long n_rows)
{
    g_log << "-> Minimizaton" << "\n";
    const std::string base = out_dir(args) + add_segment_to_filename(file_base(args["infile"]), segment) +
                             outfile_param_code(P);
    const std::string outfile_ll = base + "_iterations.csv";
    g_iter = std::ofstream(outfile_ll, std::ios_base::app);
    {   // setup_outfile_likelihood (likelihood.h:290-299)
        P.to_csv(outfile_ll);
        std::ofstream file(outfile_ll, std::ios_base::app);
        file << "\nlog_likelihoods:\niteration,";
        for (int i = 0; i < GGP_N_PARAMS; ++i) file << P.name(i) << ",";
        file << "log_likelihood" << "\n";
    }
    g_log << "Outfile: " << outfile_ll << "\n";
    const double tol = std::stod(args["tolerance_maximization"]);
    const double ll_max = minimize(o, P, tol, args["search_space"] == "log");
    g_iter.close();

    g_log << "-> Error estimation" << "\n";
    const std::string outfile_estim = base + "_final.csv";
    g_log << "Outfile: " << outfile_estim << "\n";
    P.to_csv(outfile_estim);
    {   // save_error_bars (likelihood.h:341-368)
        std::ofstream file(outfile_estim, std::ios_base::app);
        file << "\nerrors^2:";
        file << "\nepsilon";
        const std::vector<double> eps{5e-2, 1e-2, 5e-3};
        for (int i : P.non_fixed()) file << "," << P.name(i);
        file << "\n";
        for (double e : eps) {
            const std::vector<double> error = ll_error_bars(P, o, e);
            file << e;
            for (double v : error) file << "," << v;
            file << "\n";
        }
        g_clock.mark("-m: error bars (Hessians)");
    }
    {   // save_final_likelihood (likelihood.h:316-339)
        std::ofstream file(outfile_estim, std::ios_base::app);
        file << "\n";
        file << "n_data_points, " << n_rows << "\n";
        file << "total_log_likelihoood," << std::setprecision(15) << ll_max << "\n";
        file << "norm_log_likelihoood," << std::setprecision(15) << ll_max / n_rows << "\n";
        file << "optimization_algorithm," << "LN_NELDERMEAD" << "\n";
        file << "tolerance," << tol << "\n";
        file << "search_space," << args["search_space"] << "\n";
        file << "noise_model," << args["noise_model"] << "\n";
        file << "cell_division_model," << args["cell_division_model"] << "\n";
        file << "version," << "0.4.2" << "\n";
    }
    {   // create_parameter_file (likelihood.h:371-377)
        std::ofstream file(base + "_parameter_file.txt");
        file << "# Generated parameter file with the final parameters that may be used for predictions\n";
        for (int i = 0; i < GGP_N_PARAMS; ++i) file << P.name(i) << " = " << P.final_[i] << "\n";
    }
}

// ---- -s (main.cpp:80-114) ------------------------------------------------------------------
void run_bound_1dscan(Objective &o, const Params &P, std::map<std::string, std::string> &args, int segment)
{
    g_log << "-> 1d Scan" << "\n";
    g_save_ll = true;
    for (int i = 0; i < GGP_N_PARAMS; ++i) {
        if (!P.bound(i)) continue;
        std::vector<double> pv = P.get_final();
        const std::string outfile = out_dir(args) + add_segment_to_filename(file_base(args["infile"]), segment) +
                                    "_scan_" + P.name(i) + ".csv";
        g_iter = std::ofstream(outfile, std::ios_base::app);
        {
            P.to_csv(outfile);
            std::ofstream file(outfile, std::ios_base::app);
            file << "\nlog_likelihoods:\niteration,";
            for (int k = 0; k < GGP_N_PARAMS; ++k) file << P.name(k) << ",";
            file << "log_likelihood" << "\n";
        }
        g_log << "Outfile: " << outfile << "\n";
        std::vector<double> pts;   // the scan's calls, chained as the reference makes them
        for (double v : arange<double>(P.p.lower[i], P.p.upper[i], P.p.step[i])) {
            pv[i] = v;
            pts.insert(pts.end(), pv.begin(), pv.end());
        }
        total_likelihood_chain(pts, o);
    }
    g_save_ll = false;
}

// ---- -p (main.cpp:117-146, predictions.h:522-601) -----------------------------------------
void run_prediction(const ggp_dataset *d, std::vector<Params> &plist, std::map<std::string, std::string> &args)
{
    g_log << "-> prediction" << "\n";
    std::string outfile = out_dir(args) + file_base(args["infile"]);
    for (const Params &P : plist) outfile += outfile_param_code(P);
    outfile += "_prediction.csv";
    Forest F;
    g_clock.mark("-p: start");
    build_forest(F, d, -1, args["noise_model"], args["cell_division_model"]);
    g_clock.mark("-p: forest built, on device");
    std::vector<double> pv;
    for (const Params &P : plist) {
        const auto v = P.get_final();
        pv.insert(pv.end(), v.begin(), v.end());
    }
    const int64_t nr = F.desc.n_rows, nc = F.desc.n_cells;
    // the combined rows stay in HBM; the writer streams them by row ranges (bounded host memory)
    const int rc = ggp_predict(F.gpu, pv.data(), (int32_t)plist.size(), nullptr, nullptr, nullptr);
    if (rc != GGP_OK) throw std::runtime_error(std::string("ggp_predict: ") + ggp_strerror(rc));
    g_clock.mark("-p: smoother (GPU)");
    // rows per device-to-host copy (GGP_PREDICT_SPAN: a test knob; two host buffers of this many rows)
    const char *span_env = std::getenv("GGP_PREDICT_SPAN");
    const int64_t span = span_env && std::atoll(span_env) > 0 ? std::atoll(span_env) : (int64_t)1 << 20;
    std::vector<double> comb((size_t)std::min<int64_t>(span, std::max<int64_t>(nr, 1)) * 20);
    if (args.count("predict_binary")) {
        // additive: the same 4 means + 10 upper-triangle covariances per row as the CSV, in input
        // order, as raw doubles: "GGPP0001", int64 n_rows, then [n_rows x 14] f64
        const std::string binfile = outfile.substr(0, outfile.size() - 4) + ".bin";
        g_log << "Outfile: " << binfile << "\n";
        std::ofstream bf(binfile, std::ios::binary);
        bf.write("GGPP0001", 8);
        bf.write(reinterpret_cast<const char *>(&nr), 8);
        std::vector<double> row14;
        for (int64_t lo = 0; lo < nr; lo += span) {
            const int64_t hi = std::min(nr, lo + span);
            const int rr = ggp_predict_rows(F.gpu, lo, hi, comb.data());
            if (rr != GGP_OK) throw std::runtime_error(std::string("ggp_predict_rows: ") + ggp_strerror(rr));
            row14.resize((size_t)(hi - lo) * 14);
            for (int64_t r = lo; r < hi; ++r) {
                const double *s = &comb[(size_t)(r - lo) * 20];
                double *o = &row14[(size_t)(r - lo) * 14];
                for (int k = 0; k < 4; ++k) o[k] = s[k];
                int q = 4;
                for (int m = 0; m < 4; ++m)
                    for (int n = m; n < 4; ++n) o[q++] = s[4 + 4 * m + n];
            }
            bf.write(reinterpret_cast<const char *>(row14.data()), (std::streamsize)(row14.size() * sizeof(double)));
        }
        if (!bf) throw std::runtime_error("write failed: " + binfile);
        g_clock.mark("-p: binary rows written");
        return;
    }
    g_log << "Outfile: " << outfile << "\n";
    for (size_t i = 0; i < plist.size(); ++i) {
        if (i == 0)
            plist[i].to_csv(outfile);
        else
            plist[i].to_csv(outfile, std::ios_base::app);
    }
    std::ofstream file(outfile, std::ios_base::app);
    file << "\ncell_id,parent_id,time,log_length,fp,";
    file << "mean_x,mean_g,mean_l,mean_q," << "cov_xx,cov_xg,cov_xl,cov_xq," << "cov_gg,cov_gl,cov_gq,"
         << "cov_ll,cov_lq," << "cov_qq\n";
    // one line per row, cells in input order and rows in time order: rows 0..nr-1 (row_offset is
    // monotone).  Each fetched span is cut into blocks of rows formatted on every core
    // (ggp_text.h: the same bytes as the reference's `<<`), written in order; the next span is
    // copied from the device meanwhile (two host buffers; one thread calls the engine at a time).
    const int64_t *ro = F.desc.row_offset;
    const int64_t blk = 4096;
    std::vector<double> comb2(comb.size());
    std::vector<double> *buf[2] = {&comb, &comb2};
    auto fetch = [&](int64_t lo, std::vector<double> *b) {
        return nr > 0 ? ggp_predict_rows(F.gpu, lo, std::min(nr, lo + span), b->data()) : GGP_OK;
    };
    int fr = fetch(0, buf[0]);
    std::string fmsg = fr == GGP_OK ? "" : ggp_strerror(fr);   // the engine's message is per thread
    for (int64_t lo = 0, k = 0; lo < nr; lo += span, ++k) {
        if (fr != GGP_OK) throw std::runtime_error("ggp_predict_rows: " + fmsg);
        const int64_t hi = std::min(nr, lo + span);
        const double *rows = buf[k & 1]->data();
        std::thread next;
        if (hi < nr)
            next = std::thread([&, hi, k] {
                fr = fetch(hi, buf[(k + 1) & 1]);
                if (fr != GGP_OK) fmsg = ggp_strerror(fr);   // read on the thread that set it
            });
        struct Join {   // the prefetch joins on every way out of this span (a throw included)
            std::thread &t;
            ~Join()
            {
                if (t.joinable()) t.join();
            }
        } join_next{next};
        ggp_text::write_ordered(file, (hi - lo + blk - 1) / blk, [&](int64_t b, std::string &sbuf) {
            ggp_text::Sink out(sbuf);
            const int64_t r0 = lo + b * blk, r1 = std::min(hi, r0 + blk);
            int64_t c = std::upper_bound(ro, ro + nc + 1, r0) - ro - 1;   // the cell of row r0
            for (int64_t r = r0; r < r1; ++r) {
                while (r >= ro[c + 1]) ++c;
                out.str(ggp_host_forest_cell_id(F.host, c));
                out.ch(',');
                out.str(ggp_host_forest_parent_id(F.host, c));
                out.ch(',');
                out.num(F.desc.time[r]);
                out.ch(',');
                out.num(F.desc.log_length[r]);
                out.ch(',');
                out.num(F.desc.fp[r]);
                out.ch(',');
                const double *sr = rows + (size_t)(r - lo) * 20;
                out.values(sr, 4);   // the 4 means
                out.ch(',');
                out.upper(sr + 4, 4);   // output_upper_triangle
                out.ch('\n');
            }
        });
    }
    if (!file) throw std::runtime_error("write failed: " + outfile);
    g_clock.mark("-p: csv rows written");
}

// ---- -j (main.cpp:150-186; correlation_tree.h:9-23, 96-126, 588-648, 786-791) -------------
// The reference writes one dense line per start row (cells in input order, rows in time
// order): for every row of the forest -- a column, labelled cell_id_time -- either the joint
// P(z_column, z_start | D) as 8 means and the 36-entry upper triangle of its covariance, or
// 44 empty fields.  Joint_vector::add stores a joint in every column whose (cell_id, time)
// equals the target's, the last add winning.  The joints come from the GPU (ggp_joints) in
// the reference's add order, a bounded range of start rows per call, packed as they are printed
// (ggp_joints_packed: the 8 means and the covariance's upper triangle).
void write_commas(std::ostream &file, int64_t count)
{
    static const std::string block(44 * 1024, ',');
    while (count > 0) {
        const int64_t k = std::min<int64_t>(count, (int64_t)block.size());
        file.write(block.data(), (std::streamsize)k);
        count -= k;
    }
}

void run_joints(const ggp_dataset *d, std::vector<Params> &plist, std::map<std::string, std::string> &args)
{
    g_log << "-> joint posteriors" << "\n";
    std::string outfile = out_dir(args) + file_base(args["infile"]);
    for (const Params &P : plist) outfile += outfile_param_code(P);
    outfile += "_joints.csv";
    Forest F;
    build_forest(F, d, -1, args["noise_model"], args["cell_division_model"]);
    std::vector<double> pv;
    for (const Params &P : plist) {
        const auto v = P.get_final();
        pv.insert(pv.end(), v.begin(), v.end());
    }
    const double tol = std::stod(args["rel_tolerance_joints"]);
    const int64_t nr = F.desc.n_rows, nc = F.desc.n_cells;
    const double *time = F.desc.time;
    std::vector<int64_t> row_cell((size_t)nr);
    for (int64_t c = 0; c < nc; ++c)
        for (int64_t r = F.desc.row_offset[c]; r < F.desc.row_offset[c + 1]; ++r) row_cell[(size_t)r] = c;
    // columns sharing a (cell_id, time) key: get_column_indices + Joint_vector::add
    std::vector<int32_t> dup((size_t)nr, -1);
    std::vector<std::vector<int64_t>> groups;
    {
        std::unordered_map<std::string, int64_t> first;
        first.reserve((size_t)nr);
        for (int64_t r = 0; r < nr; ++r) {
            const double t = time[r] + 0.0;   // -0 == +0, as the reference's double == compares
            std::string key = ggp_host_forest_cell_id(F.host, row_cell[(size_t)r]);
            key.push_back('\0');
            key.append(reinterpret_cast<const char *>(&t), sizeof t);
            const auto ins = first.emplace(std::move(key), r);
            if (ins.second) continue;
            const int64_t f0 = ins.first->second;
            if (dup[(size_t)f0] < 0) {
                dup[(size_t)f0] = (int32_t)groups.size();
                groups.push_back({f0});
            }
            dup[(size_t)r] = dup[(size_t)f0];
            groups[(size_t)dup[(size_t)f0]].push_back(r);
        }
    }
    // additive (-js): the sparse form -- one line per (start row, column) a joint lands in, in
    // the reference's add order, the same 44 value fields; O(joints) instead of O(rows^2).
    // gfp_gaussian_process_amd/joints_format.py rebuilds the dense file from it byte for byte.
    const bool sparse = args.count("joints_sparse") > 0;
    if (sparse) outfile = outfile.substr(0, outfile.size() - 4) + "_sparse.csv";
    g_log << "Outfile: " << outfile << "\n";
    std::ofstream file(outfile);
    for (const Params &P : plist) P.to_csv(file);   // setup_outfile_joints
    if (sparse) {
        file << "\nstart_row,column,mean_0,mean_1,mean_2,mean_3,mean_4,mean_5,mean_6,mean_7,cov_upper_triangle";
        for (int k = 0; k < 35; ++k) file << ",";
        file << "\n";
    } else {
        file << "\ncell_id,parent_id,time";
        file << ",";                                 // write_column_indices
        for (int64_t r = 0; r < nr; ++r) {
            file << ggp_host_forest_cell_id(F.host, row_cell[(size_t)r]) << '_' << time[r];
            write_commas(file, r == nr - 1 ? 43 : 44);
        }
        file << "\n";
    }
    const int64_t max_cap = (int64_t)1 << 21;        // joints per call (44 doubles each: ggp_joints_packed)
    int64_t cap = (int64_t)1 << 14, chunk = 4096, chunk_max = 65536;
    std::vector<int64_t> idx((size_t)(2 * cap));
    std::vector<double> val((size_t)(44 * cap));
    int64_t logged = -1;
    for (int64_t lo = 0; lo < nr;) {
        const int64_t hi = std::min(nr, lo + chunk), s_lo = lo;
        int64_t n_out = 0;
        const int rc = ggp_joints_packed(F.gpu, pv.data(), (int32_t)plist.size(), tol, lo, hi, cap, idx.data(),
                                         val.data(), &n_out);
        if (rc == GGP_ENOMEM && hi - lo > 1) {   // the range's walk stack or slots do not fit: a smaller range
            chunk = chunk_max = std::max<int64_t>(1, (hi - lo) / 2);
            continue;
        }
        if (rc != GGP_OK) throw std::runtime_error(std::string("ggp_joints: ") + ggp_strerror(rc));
        if (n_out > cap) {   // buffers too small: split the range, or grow them
            if (n_out > max_cap && hi - lo > 1) {
                chunk = std::max<int64_t>(1, (hi - lo) / 2);
            } else {
                cap = n_out;
                idx.resize((size_t)(2 * cap));
                val.resize((size_t)(44 * cap));
            }
            continue;
        }
        // the joints of start row s are idx/val[first[s - lo], first[s - lo + 1]) (the engine emits
        // them by start row, in add order)
        std::vector<int64_t> first((size_t)(hi - lo + 1));
        {
            int64_t k = 0;
            for (int64_t s = lo; s < hi; ++s) {
                first[(size_t)(s - lo)] = k;
                while (k < n_out && idx[(size_t)(2 * k)] == s) ++k;
                const int64_t c = row_cell[(size_t)s];
                if (c != logged) {
                    g_log << "-> cell: " << c << "\n";
                    logged = c;
                }
            }
            first[(size_t)(hi - lo)] = k;
            if (k != n_out) throw std::runtime_error("ggp_joints: joints out of start-row order");
        }
        // sc_joint_distributions: one line per start row (dense), or one per (start row, column)
        // (sparse); blocks of start rows formatted on every core, written in order (ggp_text.h)
        const int64_t sblk = sparse ? 64 : 4;
        ggp_text::write_ordered(file, (hi - lo + sblk - 1) / sblk, [&](int64_t bi, std::string &buf) {
            ggp_text::Sink out(buf);
            std::map<int64_t, int64_t> cols;   // column -> joint, the last add wins
            const int64_t s0 = lo + bi * sblk, s1 = std::min(hi, s0 + sblk);
            for (int64_t s = s0; s < s1; ++s) {
                const int64_t k0 = first[(size_t)(s - lo)], k1 = first[(size_t)(s - lo + 1)];
                if (sparse) {   // every column the add reaches, in add order
                    for (int64_t k = k0; k < k1; ++k) {
                        const int64_t tgt = idx[(size_t)(2 * k + 1)];
                        const double *j = &val[(size_t)(44 * k)];   // means, then the upper triangle
                        auto line = [&](int64_t col) {
                            out.i64(s);
                            out.ch(',');
                            out.i64(col);
                            out.ch(',');
                            out.values(j, 44);
                            out.ch('\n');
                        };
                        if (dup[(size_t)tgt] < 0)
                            line(tgt);
                        else
                            for (int64_t col : groups[(size_t)dup[(size_t)tgt]]) line(col);
                    }
                    continue;
                }
                cols.clear();
                for (int64_t k = k0; k < k1; ++k) {
                    const int64_t tgt = idx[(size_t)(2 * k + 1)];
                    if (dup[(size_t)tgt] < 0)
                        cols[tgt] = k;
                    else
                        for (int64_t col : groups[(size_t)dup[(size_t)tgt]]) cols[col] = k;
                }
                const int64_t c = row_cell[(size_t)s];
                out.str(ggp_host_forest_cell_id(F.host, c));
                out.ch(',');
                out.str(ggp_host_forest_parent_id(F.host, c));
                out.ch(',');
                out.num(time[s]);
                int64_t prev = 0;
                for (const auto &e : cols) {             // Joint_vector::write
                    out.fill((size_t)(44 * (e.first - prev)), ',');
                    const double *j = &val[(size_t)(44 * e.second)];   // means, then the upper triangle
                    out.ch(',');
                    out.values(j, 44);
                    prev = e.first + 1;
                }
                out.fill((size_t)(44 * (nr - prev)), ',');
                out.ch('\n');
            }
        });
        lo = hi;
        // the next range sized for about max_cap / 2 joints at this range's density: a launch walks
        // its start rows side by side (one lane each) and takes as long as its longest walk, so
        // fewer, larger ranges mean fewer launches (up to 65,536 start rows, one wave per SIMD)
        if (n_out > 0) {
            chunk = std::min<int64_t>(chunk_max, std::max<int64_t>(std::min<int64_t>(256, chunk_max),
                                                                  (hi - s_lo) * (max_cap / 2) / n_out));
            const int64_t want = std::min<int64_t>(max_cap, (int64_t)((double)n_out * chunk / (hi - s_lo) * 1.25) + 1);
            if (want > cap) {
                cap = want;
                idx.resize((size_t)(2 * cap));
                val.resize((size_t)(44 * cap));
            }
        }
    }
    if (!file) throw std::runtime_error("write failed: " + outfile);
}

// ---- main.cpp:148-345 arg_parser ------------------------------------------------------------
std::map<std::string, std::string> arg_parser(int argc, char **argv)
{
    const std::vector<std::vector<std::string>> keys = {
        {"-h", "--help", "this help message"},
        {"-i", "--infile", "(required) input data file"},
        {"-b", "--parameter_bounds", "(required) file(s) setting the type, step, bounds of the parameters"},
        {"-c", "--csv_config", "file that sets the columns that will be used from the input file"},
        {"-l", "--print_level", "print level {0,1,2}, default: 0"},
        {"-o", "--outdir", "specify output direction and do not use default"},
        {"-t", "--tolerance_maximization", "absolute tolerance of maximization between optimization steps, default: 1e-10"},
        {"-r", "--rel_tolerance_joints", "relative tolerance of joint calculation: default 1e-10"},
        {"-space", "--search_space", "search parameter space in {'log'|'linear'} space, default: 'log'"},
        {"-noise", "--noise_model", "measurement noise of fp content {'scaled'|'const'} default: 'scaled'"},
        {"-div", "--cell_division_model", "cell divison model {'binomial'|'gauss'} default: 'binomial'"},
        {"-m", "--maximize", "run maximization"},
        {"-s", "--scan", "run 1d parameter scan"},
        {"-p", "--predict", "run prediction"},
        {"-j", "--joints", "run calculation of joint probabilities"},
        {"-e", "--evaluate", "evaluate the total log likelihood once at the parameter files' values"},
        {"-hb", "--batched_hessian", "error bars from one batched GPU call (points not chained by carried state)"},
        {"-g", "--gpus", "GPUs to shard the forest over: 'all' (default), a count N, or ordinals '0,1,..' (repeats: logical shards)"},
        {"-js", "--joints_sparse", "-j with one line per joint (_joints_sparse.csv) instead of the dense matrix"},
        {"-pbin", "--predict_binary", "write -p's rows as raw doubles (_prediction.bin) instead of the CSV"},
        {"-chunk", "--max_shard_rows", "at most this many rows per shard (caps the -p device workspace), default: one shard per GPU"},
    };
    std::map<std::string, std::string> a;
    a["print_level"] = "0";
    a["tolerance_maximization"] = "1e-10";
    a["rel_tolerance_joints"] = "1e-10";
    a["search_space"] = "log";
    a["noise_model"] = "scaled";
    a["cell_division_model"] = "binomial";
    for (size_t k = 0; k < keys.size(); ++k) {
        for (int i = 1; i < argc; ++i) {
            const std::string arg = argv[i];
            if (arg != keys[k][0] && arg != keys[k][1]) continue;
            const std::string &key = keys[k][0];
            auto next = [&]() -> std::string {
                if (i + 1 >= argc) throw std::invalid_argument("Invalide argument");
                return argv[i + 1];
            };
            if (key == "-i") a["infile"] = next();
            else if (key == "-b") {
                for (int j = i + 1; j < argc; ++j) {
                    const std::string argj = argv[j];
                    if (argj.rfind("-", 0) == 0) break;
                    a["parameter_bounds"] += argj + " ";
                }
                a["parameter_bounds"] = trim(a["parameter_bounds"]);
            } else if (key == "-c") a["csv_config"] = next();
            else if (key == "-l") a["print_level"] = next();
            else if (key == "-o") a["outdir"] = next();
            else if (key == "-t") a["tolerance_maximization"] = next();
            else if (key == "-r") a["rel_tolerance_joints"] = next();
            else if (key == "-space") a["search_space"] = next();
            else if (key == "-noise") a["noise_model"] = next();
            else if (key == "-div") a["cell_division_model"] = next();
            else if (key == "-m") a["minimize"] = "1";
            else if (key == "-s") a["scan"] = "1";
            else if (key == "-p") a["predict"] = "1";
            else if (key == "-e") a["evaluate"] = "1";
            else if (key == "-hb") a["batched_hessian"] = "1";
            else if (key == "-g") a["gpus"] = next();
            else if (key == "-chunk") a["max_shard_rows"] = next();
            else if (key == "-js") {
                a["joints"] = "1";
                a["joints_sparse"] = "1";
                a["predict"] = "1";
            } else if (key == "-pbin") {
                a["predict_binary"] = "1";
                a["predict"] = "1";
            }
            else if (key == "-j") {
                a["joints"] = "1";
                a["predict"] = "1";
            } else if (key == "-h") {
                a["help"] = "1";
                std::cout << "Usage: ./gfp_gaussian [-options]\n";
                for (const auto &kk : keys) std::cout << pad_str(kk[0] + ", " + kk[1], 35) << kk[2] << "\n";
            }
        }
    }
    if (a.count("help")) return a;
    if (a["search_space"] != "log" && a["search_space"] != "linear") {
        std::cout << "(arg_parser) ERROR: search_space must be either 'log' or 'linear', not " << a["search_space"];
        throw std::invalid_argument("Invalide argument");
    }
    if (a["noise_model"] != "const" && a["noise_model"] != "scaled") {
        std::cout << "(arg_parser) ERROR: noise_model must be either 'const' or 'scaled', not " << a["noise_model"];
        throw std::invalid_argument("Invalide argument");
    }
    if (a["cell_division_model"] != "gauss" && a["cell_division_model"] != "binomial") {
        std::cout << "(arg_parser) ERROR: cell_division_model must be either 'gauss' or 'binomial', not "
                  << a["cell_division_model"];
        throw std::invalid_argument("Invalide argument");
    }
    if (!a.count("infile")) {
        std::cout << "(arg_parser) ERROR: Required infile flag not set!\n";
        throw std::invalid_argument("Invalide argument");
    } else if (!std::filesystem::exists(a["infile"])) {
        std::cout << "(arg_parser) ERROR: Infile " << a["infile"] << " not found (use '-h' for help)!" << std::endl;
        throw std::invalid_argument("Invalide argument");
    }
    if (!a.count("parameter_bounds")) {
        std::cout << "(arg_parser) ERROR: Required parameter_bounds flag not set!\n";
        throw std::invalid_argument("Invalide argument");
    }
    for (const auto &pf : split_string_at(a["parameter_bounds"], " ")) {
        if (!std::filesystem::exists(pf)) {
            std::cout << "(arg_parser) ERROR: Paramters bound file '" << pf << "' not found (use '-h' for help)!"
                      << std::endl;
            throw std::invalid_argument("Invalide argument");
        }
    }
    if (a.count("csv_config") && !std::filesystem::exists(a["csv_config"])) {
        std::cout << "(arg_parser) ERROR: csv_config flag set, but csv configuration file " << a["csv_config"]
                  << " not found!" << std::endl;
        throw std::invalid_argument("Invalide argument");
    }
    return a;
}

}  // namespace

int main(int argc, char **argv)
{
    std::string outfile_log, outfile_log_success, outfile_log_error;
    std::cout << "Running... \n";
    ggp_dataset *data = nullptr;
    ggp_csv_config *cfg = nullptr;
    try {
        auto args = arg_parser(argc, argv);
        g_print_level = std::stoi(args["print_level"]);
        if (args.count("help")) return EXIT_SUCCESS;
        const std::string base = out_dir(args) + file_base(args["infile"]);
        outfile_log = base + ".log";
        outfile_log_success = base + "_success.log";
        outfile_log_error = base + "_error.log";

        const auto param_files = split_string_at(args["parameter_bounds"], " ");
        std::vector<Params> plist;
        g_log = std::ofstream(outfile_log, std::ios_base::app);
        std::cout << "Temporary log file '" << outfile_log << "' created\n";
        for (const auto &pf : param_files) {
            Params P;
            if (ggp_param_file_load(pf.c_str(), 1, &P.p) != GGP_OK) {
                g_log << ggp_host_last_error() << "\n";
                throw std::invalid_argument("Invalide argument");
            }
            g_log << P << "\n";
            plist.push_back(P);
        }

        const char *cfg_path = args.count("csv_config") ? args["csv_config"].c_str() : "";
        if (ggp_csv_config_load(cfg_path, &cfg) != GGP_OK) throw std::invalid_argument(ggp_host_last_error());
        g_log << "-> Reading" << "\n";
        if (ggp_dataset_is_binary(args["infile"].c_str())) {   // additive: a GGPD0001 binary dataset
            if (ggp_dataset_load(args["infile"].c_str(), &data) != GGP_OK)
                throw std::invalid_argument(ggp_host_last_error());
        } else if (ggp_dataset_read(args["infile"].c_str(), cfg, &data) != GGP_OK) {
            throw std::invalid_argument(ggp_host_last_error());
        }
        g_clock.mark("read the input");
        int32_t nseg = 0;
        ggp_dataset_segments(data, nullptr, 0, &nseg);
        std::vector<int32_t> seg(nseg);
        ggp_dataset_segments(data, seg.data(), nseg, &nseg);
        if ((size_t)nseg != param_files.size()) {
            g_log << "(main) ERROR: There are " << nseg << " segments, but " << param_files.size()
                  << " parameter files!\n";
            throw std::invalid_argument("Invalide argument");
        }
        auto file_number = [&](int i) { return nseg > 1 ? i : -1; };

        g_batched_hessian = args.count("batched_hessian") > 0;
        if (args.count("gpus") && args["gpus"] != "all") {
            const std::string gs = args["gpus"];
            if (gs.find(',') == std::string::npos) {
                const int n = std::stoi(gs);
                if (n < 1) throw std::invalid_argument("Invalide argument");
                for (int k = 0; k < n; ++k) g_devices.push_back(k);
            } else {
                for (const auto &t : split_string_at(gs, ","))
                    if (!t.empty()) g_devices.push_back(std::stoi(t));
            }
        }
        if (args.count("max_shard_rows")) g_max_shard_rows = std::stoll(args["max_shard_rows"]);
        if (args.count("evaluate")) {
            for (int i = 0; i < nseg; ++i) {
                Forest F;
                build_forest(F, data, seg[i], args["noise_model"], args["cell_division_model"]);
                Objective o{F.gpu, F.host, &F.desc};
                const double ll = total_likelihood(plist[i].get_final(), o);
                std::cout << "segment " << seg[i] << ": total log likelihood = " << std::setprecision(17) << ll
                          << " (" << F.desc.n_rows << " data points)\n";
                g_log << "total log likelihood (segment " << seg[i] << ") = " << std::setprecision(17) << ll << "\n";
            }
        }
        if (args.count("minimize")) {
            for (int i = 0; i < nseg; ++i) {
                if (!plist[i].has_nonfixed()) continue;
                Forest F;
                build_forest(F, data, seg[i], args["noise_model"], args["cell_division_model"]);
                Objective o{F.gpu, F.host, &F.desc};
                run_minimization(o, plist[i], args, file_number(i), (long)F.desc.n_rows);
            }
        }
        if (args.count("scan")) {
            for (int i = 0; i < nseg; ++i) {
                Forest F;
                build_forest(F, data, seg[i], args["noise_model"], args["cell_division_model"]);
                Objective o{F.gpu, F.host, &F.desc};
                run_bound_1dscan(o, plist[i], args, file_number(i));
            }
        }
        if (args.count("predict")) run_prediction(data, plist, args);
        if (args.count("joints")) run_joints(data, plist, args);   // after -p (main.cpp:440-443)

        g_log << "Done." << std::endl;
        std::cout << "Done. Log file: " << outfile_log_success << std::endl;
        std::rename(outfile_log.c_str(), outfile_log_success.c_str());
        g_log.close();
        ggp_dataset_free(data);
        ggp_csv_config_free(cfg);
        return EXIT_SUCCESS;
    } catch (std::exception &e) {
        if (!outfile_log.empty()) std::rename(outfile_log.c_str(), outfile_log_error.c_str());
        g_log << "Quit because of an error: " << e.what() << "\n";
        g_log.close();
        std::cout << "Quit because of an error: " << e.what() << "\n";
        std::cout << "Error log file: " << outfile_log_error << std::endl;
        if (data) ggp_dataset_free(data);
        if (cfg) ggp_csv_config_free(cfg);
        return EXIT_FAILURE;
    }
}
