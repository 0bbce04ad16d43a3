// ggp_text.h -- the CLI's bulk text output (-p _prediction.csv, -j / -js joints) formatted on
// every host core, written in order.
//
// The reference streams every number through `std::ostream << double` with the default
// formatting (predictions.h:540-602, correlation_tree.h:96-126): precision 6, no floatfield,
// which libstdc++ renders as printf's "%.6g".  std::to_chars(general, 6) is specified as that
// same printf conversion, so put_num() appends byte-for-byte what `<<` would have written, with
// no locale or stream state per number (tests/test_host.py checks it against an ostringstream
// and against Python's '%.6g' on a million values, NaN, inf, signed zero and subnormals).
//
// At C5 the prediction file is ~100 GB of text: one formatting thread runs at
// ~0.1-0.2 GB/s, so the rows of a range are cut into blocks, the blocks formatted into strings
// by a pool of threads, and the strings written in block order -- the file is the serial one.
#pragma once
#include <algorithm>
#include <atomic>
#include <charconv>
#include <condition_variable>
#include <cstdint>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <ostream>
#include <string>
#include <thread>
#include <vector>

namespace ggp_text {

// 10^k, k = -308..308, as doubles (exact for |k| <= 22, rounded beyond)
struct Pow10 {
    double v[617];
    Pow10()
    {
        v[308] = 1.0;
        long double p = 1.0L;
        for (int k = 1; k <= 308; ++k) {
            p *= 10.0L;
            v[308 + k] = (double)p;
        }
        p = 1.0L;
        for (int k = 1; k <= 308; ++k) {
            p /= 10.0L;
            v[308 - k] = (double)p;
        }
        for (int k = 0; k <= 22; ++k) {   // the exact ones exactly
            double q = 1.0;
            for (int j = 0; j < k; ++j) q *= 10.0;
            v[308 + k] = q;
        }
    }
    double operator()(int k) const { return v[308 + k]; }
};
inline const Pow10 &pow10_table()
{
    static const Pow10 t;
    return t;
}

// "%.6g" of x into b (at least 32 bytes); returns the end.  Fast path: |x| in [1e-290, 1e290]
// scaled into [1e5, 1e6) by a power of ten (a few ulp of error, < 1e-9 absolute) and rounded to
// the nearest integer -- the six significant digits -- whenever the fraction is more than 1e-8
// away from one half, i.e. whenever that error cannot change the rounding.  Everything else (0,
// subnormals, inf, NaN, huge values, near-ties) goes through std::to_chars(general, 6), which is
// printf's exact conversion.
inline char *fmt_g6(char *b, double x)
{
    const double ax = x < 0 ? -x : x;
    if (ax >= 1e-290 && ax <= 1e290) {
        const Pow10 &P = pow10_table();
        uint64_t bits;
        std::memcpy(&bits, &ax, 8);
        const int e2 = (int)(bits >> 52) - 1023;
        int e = (e2 * 78913) >> 18;   // floor(e2 log10 2): floor(log10 ax) or one below
        double sc = ax * P(5 - e);
        if (sc >= 1e6) {
            ++e;
            sc = ax * P(5 - e);
        }
        const double fl = (double)(int64_t)sc;   // sc > 0: truncation is floor
        const double fr = sc - fl;
        if (fl >= 99999.0 && fl < 1e6 && (fr < 0.5 - 1e-8 || fr > 0.5 + 1e-8)) {
            uint32_t d = (uint32_t)fl + (fr > 0.5 ? 1u : 0u);
            if (d < 100000) {   // the value is below 1e5 x 10^(e-5): one decade down
                --e;
                sc = ax * P(5 - e);
                const double f2 = (double)(int64_t)sc, r2 = sc - f2;
                if (!(r2 < 0.5 - 1e-8 || r2 > 0.5 + 1e-8)) goto slow;
                d = (uint32_t)f2 + (r2 > 0.5 ? 1u : 0u);
            }
            if (d == 1000000) {
                d = 100000;
                ++e;
            }
            if (d < 100000 || d >= 1000000) goto slow;
            char dg[6];
            for (int i = 5; i >= 0; --i) {
                dg[i] = (char)('0' + d % 10);
                d /= 10;
            }
            int nd = 6;   // significant digits without trailing zeros
            while (nd > 1 && dg[nd - 1] == '0') --nd;
            char *o = b;
            if (x < 0) *o++ = '-';
            if (e >= -4 && e < 6) {   // fixed
                if (e >= 0) {
                    for (int i = 0; i <= e; ++i) *o++ = i < nd ? dg[i] : '0';
                    if (nd > e + 1) {
                        *o++ = '.';
                        for (int i = e + 1; i < nd; ++i) *o++ = dg[i];
                    }
                } else {
                    *o++ = '0';
                    *o++ = '.';
                    for (int i = 0; i < -e - 1; ++i) *o++ = '0';
                    for (int i = 0; i < nd; ++i) *o++ = dg[i];
                }
            } else {   // scientific: d.ddddde+XX
                *o++ = dg[0];
                if (nd > 1) {
                    *o++ = '.';
                    for (int i = 1; i < nd; ++i) *o++ = dg[i];
                }
                *o++ = 'e';
                *o++ = e < 0 ? '-' : '+';
                const int ae = e < 0 ? -e : e;
                if (ae >= 100) *o++ = (char)('0' + ae / 100);
                *o++ = (char)('0' + ae / 10 % 10);
                *o++ = (char)('0' + ae % 10);
            }
            return o;
        }
    }
slow:
#ifdef GGP_TEXT_COUNT_SLOW
    GGP_TEXT_COUNT_SLOW;
#endif
    return std::to_chars(b, b + 32, x, std::chars_format::general, 6).ptr;
}

// `os << x` for a double under the default stream state ("%.6g")
inline void put_num(std::string &s, double x)
{
    char b[32];
    s.append(b, fmt_g6(b, x));
}

inline void put_int(std::string &s, int64_t v)
{
    char b[24];
    const auto r = std::to_chars(b, b + sizeof b, v);
    s.append(b, r.ptr);
}

// Appends to a std::string through a raw cursor (no per-number append call): the string grows
// geometrically, and is cut to the bytes written when the Sink goes out of scope.
class Sink {
public:
    explicit Sink(std::string &s) : s_(s), n_(s.size()) {}
    ~Sink() { s_.resize(n_); }
    Sink(const Sink &) = delete;
    Sink &operator=(const Sink &) = delete;

    void num(double x)   // `<< x`
    {
        char *p = room(32);
        n_ = (size_t)(fmt_g6(p, x) - s_.data());
    }
    void i64(int64_t v)
    {
        char *p = room(24);
        n_ = (size_t)(std::to_chars(p, p + 24, v).ptr - s_.data());
    }
    void ch(char c) { *room(1) = c, ++n_; }
    void fill(size_t k, char c)
    {
        std::memset(room(k), c, k);
        n_ += k;
    }
    void str(const char *z)
    {
        const size_t k = std::strlen(z);
        std::memcpy(room(k), z, k);
        n_ += k;
    }
    // v[0..n) comma-separated (output_vector, predictions.h:553-560)
    void values(const double *v, int n)
    {
        for (int k = 0; k < n; ++k) {
            if (k > 0) ch(',');
            num(v[k]);
        }
    }
    // the upper triangle of the row-major n x n C, row by row (output_upper_triangle,
    // predictions.h:540-551)
    void upper(const double *C, int n)
    {
        for (int m = 0; m < n; ++m)
            for (int k = m; k < n; ++k) {
                if (k + m > 0) ch(',');
                num(C[n * m + k]);
            }
    }

private:
    char *room(size_t k)
    {
        if (n_ + k > s_.size()) s_.resize(std::max<size_t>(2 * s_.size(), n_ + k + 4096));
        return &s_[n_];
    }
    std::string &s_;
    size_t n_;
};

// formatting threads: GGP_IO_THREADS, else OMP_NUM_THREADS (16 on the GPU box, whose nproc
// reports the whole machine), else the hardware's; at most 64
inline int io_threads()
{
    for (const char *var : {"GGP_IO_THREADS", "OMP_NUM_THREADS"}) {
        const char *e = std::getenv(var);
        if (e && std::atoi(e) > 0) return std::min(64, std::atoi(e));
    }
    return std::max(1, std::min(64, (int)std::thread::hardware_concurrency()));
}

// format blocks 0..n_blocks-1 with fmt(block, std::string &) on io_threads() threads and write
// them to `out` in block order as they complete (the calling thread writes while the pool
// formats).  At most `window` formatted blocks are held at once (bounded memory).  An exception
// in a formatting thread stops the pool and is rethrown here, after every thread has joined.
template <class Fmt>
void write_ordered(std::ostream &out, int64_t n_blocks, Fmt &&fmt, int64_t window = 0)
{
    if (n_blocks <= 0) return;
    const int nt = (int)std::min<int64_t>(io_threads(), n_blocks);
    if (window <= 0) window = 4 * (int64_t)nt;
    window = std::min(window, n_blocks);
    std::vector<std::string> slot((size_t)window);
    std::vector<int64_t> ready((size_t)window, -1);   // block held by the slot, once formatted
    int64_t written = 0;                             // blocks written so far
    bool stop = false;                               // a thread failed (or the writer did)
    std::exception_ptr err;
    std::atomic<int64_t> next{0};
    std::mutex mu;
    std::condition_variable cv_ready, cv_free;
    auto work = [&]() {
        for (int64_t b; (b = next.fetch_add(1)) < n_blocks;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_free.wait(lk, [&] { return stop || b - written < window; });
                if (stop) return;
            }
            std::string &s = slot[(size_t)(b % window)];
            try {
                s.clear();
                fmt(b, s);
            } catch (...) {
                std::lock_guard<std::mutex> lk(mu);
                if (!err) err = std::current_exception();
                stop = true;
                cv_ready.notify_all();
                cv_free.notify_all();
                return;
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                ready[(size_t)(b % window)] = b;
            }
            cv_ready.notify_one();
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(work);
    for (int64_t b = 0; b < n_blocks; ++b) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv_ready.wait(lk, [&] { return stop || ready[(size_t)(b % window)] == b; });
            if (stop) break;
        }
        const std::string &s = slot[(size_t)(b % window)];
        out.write(s.data(), (std::streamsize)s.size());
        {
            std::lock_guard<std::mutex> lk(mu);
            written = b + 1;
        }
        cv_free.notify_all();
    }
    for (auto &th : pool) th.join();
    if (err) std::rethrow_exception(err);
}

}  // namespace ggp_text
