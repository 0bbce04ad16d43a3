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
#include <cstdlib>
#include <mutex>
#include <ostream>
#include <string>
#include <thread>
#include <vector>

namespace ggp_text {

// `os << x` for a double under the default stream state ("%.6g")
inline void put_num(std::string &s, double x)
{
    char b[32];
    const auto r = std::to_chars(b, b + sizeof b, x, std::chars_format::general, 6);
    s.append(b, r.ptr);
}

inline void put_int(std::string &s, int64_t v)
{
    char b[24];
    const auto r = std::to_chars(b, b + sizeof b, v);
    s.append(b, r.ptr);
}

// v[0..n) comma-separated (output_vector, predictions.h:553-560)
inline void put_values(std::string &s, const double *v, int n)
{
    for (int k = 0; k < n; ++k) {
        if (k > 0) s.push_back(',');
        put_num(s, v[k]);
    }
}

// the upper triangle of the row-major n x n C, row by row (output_upper_triangle,
// predictions.h:540-551)
inline void put_upper(std::string &s, const double *C, int n)
{
    for (int m = 0; m < n; ++m)
        for (int k = m; k < n; ++k) {
            if (k + m > 0) s.push_back(',');
            put_num(s, C[n * m + k]);
        }
}

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
// formats).  At most `window` formatted blocks are held at once (bounded memory).
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
    std::atomic<int64_t> next{0};
    std::mutex mu;
    std::condition_variable cv_ready, cv_free;
    auto work = [&]() {
        for (int64_t b; (b = next.fetch_add(1)) < n_blocks;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_free.wait(lk, [&] { return b - written < window; });
            }
            std::string &s = slot[(size_t)(b % window)];
            s.clear();
            fmt(b, s);
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
            cv_ready.wait(lk, [&] { return ready[(size_t)(b % window)] == b; });
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
}

}  // namespace ggp_text
