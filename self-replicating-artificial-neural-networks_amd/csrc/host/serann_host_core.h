// serann_host_core.h: the algorithms of the native host runtime, free of Python so that the
// sanitizer self-test (selftest.cpp, tests/test_sanitizers.py) builds them under ASan/UBSan/TSan.
//
//  * levenshtein / levenshtein_batch -- unit-cost global edit distance (what edlib.align returns as
//    'editDistance' in the reference: evolutionary_experiment/logic/experiment.py:16-17,232-236),
//    Myers/Hyyro bit-parallel algorithm over 64-bit blocks, O(ceil(m/64) * n); the batch version
//    fans out over std::threads.
//  * genotype_pair_sums -- sum of pairwise Hamming distances and of their square roots over
//    bit-packed genotypes (scipy pdist/cdist in experiment.py:246-251), popcount based.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace serann_host {

// Myers' bit-vector algorithm, block-based (Hyyro 2003) for global (NW) distance.
inline int myers_blocks(const std::string& a, const std::string& b) {
    const std::string& p = a.size() <= b.size() ? a : b;   // pattern = shorter
    const std::string& t = a.size() <= b.size() ? b : a;
    const int m = (int)p.size(), n = (int)t.size();
    if (m == 0) return n;
    const int W = (m + 63) / 64;
    // Peq per character (bytes)
    std::vector<uint64_t> peq(256 * (size_t)W, 0ull);
    for (int i = 0; i < m; ++i) {
        unsigned char c = (unsigned char)p[i];
        peq[(size_t)c * W + i / 64] |= 1ull << (i % 64);
    }
    std::vector<uint64_t> Pv(W, ~0ull), Mv(W, 0ull);
    std::vector<int> score(W);
    for (int w = 0; w < W; ++w) score[w] = std::min(64 * (w + 1), m);
    const uint64_t lastbit = 1ull << ((m - 1) % 64);
    for (int j = 0; j < n; ++j) {
        const uint64_t* Eq = &peq[(size_t)(unsigned char)t[j] * W];
        int hin = 1;   // global alignment: top row increases by one per column
        for (int w = 0; w < W; ++w) {
            uint64_t pv = Pv[w], mv = Mv[w], eq = Eq[w];
            uint64_t hinNeg = hin < 0 ? 1ull : 0ull;
            uint64_t xv = eq | mv;
            eq |= hinNeg;
            uint64_t xh = (((eq & pv) + pv) ^ pv) | eq;
            uint64_t ph = mv | ~(xh | pv);
            uint64_t mh = pv & xh;
            const uint64_t hb = (w == W - 1) ? lastbit : (1ull << 63);
            int hout = (ph & hb) ? 1 : ((mh & hb) ? -1 : 0);
            ph <<= 1; mh <<= 1;
            mh |= hinNeg;
            if (hin > 0) ph |= 1ull;
            pv = mh | ~(xv | ph);
            mv = ph & xv;
            Pv[w] = pv; Mv[w] = mv;
            score[w] += hout;
            hin = hout;
        }
    }
    return score[W - 1];
}

inline int levenshtein(const std::string& a, const std::string& b) { return myers_blocks(a, b); }

inline std::vector<int> levenshtein_batch(const std::vector<std::string>& a, const std::vector<std::string>& b,
                                         int threads) {
    if (a.size() != b.size()) throw std::runtime_error("levenshtein_batch: size mismatch");
    const size_t n = a.size();
    std::vector<int> out(n);
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    threads = (int)std::min<size_t>((size_t)threads, std::max<size_t>(1, n / 16));
    if (threads <= 1) {
        for (size_t i = 0; i < n; ++i) out[i] = myers_blocks(a[i], b[i]);
        return out;
    }
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t]() {
            for (size_t i = t; i < n; i += threads) out[i] = myers_blocks(a[i], b[i]);
        });
    for (auto& th : pool) th.join();
    return out;
}

// bits: n rows of W packed 64-bit words.  Sums over i < j of hamming(i, j) and of sqrt(hamming).
inline void genotype_pair_sums(const uint64_t* bits, int64_t n, int64_t W, double& sum_hamming, double& sum_sqrt) {
    double sh = 0.0, se = 0.0;
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = i + 1; j < n; ++j) {
            int d = 0;
            for (int64_t w = 0; w < W; ++w) d += __builtin_popcountll(bits[i * W + w] ^ bits[j * W + w]);
            sh += d;
            se += std::sqrt((double)d);
        }
    sum_hamming = sh;
    sum_sqrt = se;
}

}  // namespace serann_host
