// text_check.cpp -- test driver for csrc/host/ggp_text.h (built and run by tests/test_text.py).
//
//   text_check formats SEED N   : N doubles (random bit patterns, decimal-scale values, specials)
//                                 through put_num and through `std::ostringstream <<`; prints the
//                                 mismatch count, then the first 2000 put_num strings, one a line
//   text_check ordered THREADS  : write_ordered over 5000 blocks of different lengths against the
//                                 same blocks concatenated serially; prints "same" or "differ"
//   text_check throws THREADS   : a formatting thread throws; write_ordered rethrows it
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "ggp_text.h"

static std::vector<double> values(uint64_t seed, int64_t n)
{
    std::mt19937_64 g(seed);
    std::vector<double> v = {0.0, -0.0, 1.0, -1.0, 1e-5, 1e-4, 0.0001234565, 123456.5, 999999.5, 1e6, 1e16,
                             std::numeric_limits<double>::infinity(), -std::numeric_limits<double>::infinity(),
                             std::numeric_limits<double>::quiet_NaN(), -std::numeric_limits<double>::quiet_NaN(),
                             std::numeric_limits<double>::denorm_min(), std::numeric_limits<double>::min(),
                             std::numeric_limits<double>::max(), -2.5e-310, 0.5, 2.5, 1.2345649999999999};
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    while ((int64_t)v.size() < n) {
        const uint64_t bits = g();
        double x;
        switch (bits % 7) {
        case 0: std::memcpy(&x, &bits, 8); break;                               // any bit pattern
        case 1: x = std::ldexp(u(g), (int)(g() % 120) - 60); break;              // the data's scales
        case 2: x = std::round(u(g) * 1e7) / std::pow(10.0, (double)(g() % 9)); break;   // short decimals
        case 3: x = (double)(int64_t)(u(g) * 1e9); break;                       // integers
        case 4: {   // near six-digit rounding ties: (n + 1/2) 10^k and its neighbours
            const double t = ((double)(100000 + g() % 900000) + 0.5) * std::pow(10.0, (double)((int)(g() % 41) - 25));
            const int s = (int)(g() % 5) - 2;
            x = t;
            for (int i = 0; i < (s < 0 ? -s : s); ++i) x = std::nextafter(x, s < 0 ? 0.0 : 1e308);
            break;
        }
        case 5: {   // decade edges: 10^k, 999999.5 10^k and neighbours
            const int k = (int)(g() % 600) - 300;
            const double t = (g() & 1) ? std::pow(10.0, (double)k) : 9.999995 * std::pow(10.0, (double)k);
            const int s = (int)(g() % 7) - 3;
            x = t;
            for (int i = 0; i < (s < 0 ? -s : s); ++i) x = std::nextafter(x, s < 0 ? 0.0 : 1e308);
            break;
        }
        default: x = std::ldexp(u(g), (int)(g() % 2100) - 1075); break;        // every binade
        }
        if (g() & 1) x = -x;
        v.push_back(x);
    }
    return v;
}

int main(int argc, char **argv)
{
    if (argc < 3) return 2;
    if (!std::strcmp(argv[1], "formats")) {
        const auto v = values(std::strtoull(argv[2], nullptr, 10), argc > 3 ? std::atoll(argv[3]) : 1000000);
        int64_t bad = 0;
        std::vector<std::string> first;
        for (double x : v) {
            std::string a;
            ggp_text::put_num(a, x);
            std::ostringstream o;
            o << x;
            if (a != o.str()) {
                if (bad < 5) std::fprintf(stderr, "mismatch: put_num %s, ostream %s\n", a.c_str(), o.str().c_str());
                ++bad;
            }
            if (first.size() < 2000) first.push_back(a);
        }
        std::printf("%" PRId64 "\n", bad);
        for (size_t i = 0; i < first.size(); ++i) {
            uint64_t bits;
            std::memcpy(&bits, &v[i], 8);
            std::printf("%016" PRIx64 " %s\n", bits, first[i].c_str());
        }
        return 0;
    }
    if (!std::strcmp(argv[1], "ordered")) {
        setenv("GGP_IO_THREADS", argv[2], 1);
        const int64_t nb = 5000;
        auto fmt = [](int64_t b, std::string &s) {
            for (int64_t k = 0; k < (b * 7919) % 97; ++k) {
                ggp_text::put_int(s, b);
                s.push_back(',');
                ggp_text::put_num(s, std::sqrt((double)(b * 131 + k)));
                s.push_back('\n');
            }
        };
        std::string serial;
        for (int64_t b = 0; b < nb; ++b) fmt(b, serial);
        std::ostringstream out;
        ggp_text::write_ordered(out, nb, fmt, 7);
        std::printf("%s\n", out.str() == serial ? "same" : "differ");
        return 0;
    }
    if (!std::strcmp(argv[1], "throws")) {   // a formatting thread throws: rethrown by write_ordered
        setenv("GGP_IO_THREADS", argv[2], 1);
        std::ostringstream out;
        try {
            ggp_text::write_ordered(out, 1000, [](int64_t b, std::string &s) {
                if (b == 377) throw std::runtime_error("block 377");
                ggp_text::put_int(s, b);
            }, 5);
        } catch (const std::runtime_error &e) {
            std::printf("caught %s\n", e.what());
            return 0;
        }
        std::printf("not thrown\n");
        return 1;
    }
    return 2;
}
