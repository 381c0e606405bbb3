// Sanitizer self-test of the native host runtime (serann_host_core.h), built and run by
// tests/test_sanitizers.py once under AddressSanitizer + UndefinedBehaviorSanitizer and once under
// ThreadSanitizer (the threaded Levenshtein batch is the runtime's only shared-memory concurrency).
//
// Checks, on seeded random inputs:
//  * myers_blocks against the O(mn) dynamic programme, across the 64-bit block boundaries
//    (lengths 0..300), high-bit bytes included;
//  * levenshtein_batch (several thread counts) against the serial distances;
//  * genotype_pair_sums against an unpacked per-bit Hamming loop.
// Prints "selftest ok ..." and exits 0, or prints the first mismatch and exits 1.
#include <cmath>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "serann_host_core.h"

static int dp_distance(const std::string& a, const std::string& b) {
    std::vector<int> prev(b.size() + 1), cur(b.size() + 1);
    for (size_t j = 0; j <= b.size(); ++j) prev[j] = (int)j;
    for (size_t i = 1; i <= a.size(); ++i) {
        cur[0] = (int)i;
        for (size_t j = 1; j <= b.size(); ++j) {
            const int sub = prev[j - 1] + (a[i - 1] == b[j - 1] ? 0 : 1);
            cur[j] = std::min(sub, std::min(prev[j], cur[j - 1]) + 1);
        }
        std::swap(prev, cur);
    }
    return prev[b.size()];
}

static std::string random_string(std::mt19937_64& rng, int len, int alphabet) {
    std::string s(len, ' ');
    for (int i = 0; i < len; ++i) {
        const int c = (int)(rng() % alphabet);
        s[i] = (char)(c < alphabet - 2 ? 'a' + c : 0xC0 + c);   // two high-bit byte values
    }
    return s;
}

// b = a with a few random edits (the regime of parent / mutant source codes)
static std::string mutate(std::mt19937_64& rng, const std::string& a, int edits, int alphabet) {
    std::string b = a;
    for (int e = 0; e < edits; ++e) {
        const int op = (int)(rng() % 3);
        const size_t pos = b.empty() ? 0 : rng() % b.size();
        const char c = random_string(rng, 1, alphabet)[0];
        if (op == 0 || b.empty()) b.insert(b.begin() + (long)pos, c);
        else if (op == 1) b.erase(b.begin() + (long)pos);
        else b[pos] = c;
    }
    return b;
}

int main() {
    std::mt19937_64 rng(20261016);
    std::vector<std::string> as, bs;
    int checked = 0;
    for (int t = 0; t < 600; ++t) {
        const int alphabet = 2 + (int)(rng() % 30);
        const int la = (int)(rng() % 301);
        std::string a = random_string(rng, la, alphabet);
        std::string b = (t % 2) ? mutate(rng, a, (int)(rng() % 12), alphabet)
                                : random_string(rng, (int)(rng() % 301), alphabet);
        const int got = serann_host::levenshtein(a, b), want = dp_distance(a, b);
        if (got != want) {
            std::printf("levenshtein mismatch: |a|=%zu |b|=%zu got %d want %d\n", a.size(), b.size(), got, want);
            return 1;
        }
        as.push_back(a);
        bs.push_back(b);
        ++checked;
    }
    const std::vector<int> serial = serann_host::levenshtein_batch(as, bs, 1);
    for (int threads : {2, 3, 8, 0}) {
        const std::vector<int> par = serann_host::levenshtein_batch(as, bs, threads);
        if (par != serial) {
            std::printf("levenshtein_batch(threads=%d) differs from the serial batch\n", threads);
            return 1;
        }
    }

    // genotype pair sums: 97 genotypes of 100 bits packed into 2 words (the last one partial)
    const int n = 97, L = 100, W = (L + 63) / 64;
    std::vector<std::vector<int>> g(n, std::vector<int>(L));
    std::vector<uint64_t> bits((size_t)n * W, 0);
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < L; ++k) {
            g[i][k] = (int)(rng() & 1);
            if (g[i][k]) bits[(size_t)i * W + k / 64] |= 1ull << (k % 64);
        }
    double sh = 0, se = 0, wh = 0, we = 0;
    serann_host::genotype_pair_sums(bits.data(), n, W, sh, se);
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j) {
            int d = 0;
            for (int k = 0; k < L; ++k) d += g[i][k] != g[j][k];
            wh += d;
            we += std::sqrt((double)d);
        }
    if (sh != wh || std::fabs(se - we) > 1e-9 * we) {
        std::printf("genotype_pair_sums mismatch: %f %f vs %f %f\n", sh, se, wh, we);
        return 1;
    }
    std::printf("selftest ok: %d edit distances, batch threads 1/2/3/8/auto, %d genotype pairs\n", checked,
                n * (n - 1) / 2);
    return 0;
}
