// serann_host: native host-side runtime helpers for SeRANN-AMD (Python bindings of
// serann_host_core.h: edit distance and genotype statistics).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include "serann_host_core.h"

namespace py = pybind11;

static int levenshtein(const std::string& a, const std::string& b) { return serann_host::levenshtein(a, b); }

static std::vector<int> levenshtein_batch(const std::vector<std::string>& a, const std::vector<std::string>& b,
                                          int threads) {
    py::gil_scoped_release release;
    return serann_host::levenshtein_batch(a, b, threads);
}

// bits: (n, words) uint64 packed genotypes.  Returns (sum over i<j of hamming, sum over i<j of
// sqrt(hamming)).
static py::tuple genotype_pair_stats(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> bits) {
    if (bits.ndim() != 2) throw std::runtime_error("genotype_pair_stats: expected a 2-D array");
    const int64_t n = bits.shape(0), W = bits.shape(1);
    double sh = 0.0, se = 0.0;
    {
        py::gil_scoped_release release;
        serann_host::genotype_pair_sums(bits.data(), n, W, sh, se);
    }
    return py::make_tuple(sh, se);
}

PYBIND11_MODULE(serann_host, m) {
    m.doc() = "SeRANN-AMD native host runtime (edit distance, genotype statistics)";
    m.def("levenshtein", &levenshtein, "unit-cost global edit distance");
    m.def("levenshtein_batch", &levenshtein_batch, py::arg("a"), py::arg("b"), py::arg("threads") = 0);
    m.def("genotype_pair_stats", &genotype_pair_stats);
}
