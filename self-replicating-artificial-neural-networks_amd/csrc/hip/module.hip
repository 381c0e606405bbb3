// pybind11 bindings of the SeRANN-AMD HIP kernels.  Pointers and streams are passed as integers
// (tensor.data_ptr(), torch.cuda.current_stream().cuda_stream) so that the module has no libtorch
// ABI dependency; it shares torch's HIP runtime (libamdhip64.so.7 is already loaded by torch).
#include <pybind11/pybind11.h>
#include "common.h"
#include "serann_hip.h"

namespace py = pybind11;

#ifndef SERANN_SRC_HASH
#define SERANN_SRC_HASH "unknown"
#endif

static py::dict desc_sizes() {
    py::dict d;
    d["GemmDesc"] = sizeof(GemmDesc);
    d["BnDesc"] = sizeof(BnDesc);
    d["PoolDesc"] = sizeof(PoolDesc);
    d["CopyDesc"] = sizeof(CopyDesc);
    d["EwDesc"] = sizeof(EwDesc);
    d["LossDesc"] = sizeof(LossDesc);
    d["TransDesc"] = sizeof(TransDesc);
    d["ImcolDesc"] = sizeof(ImcolDesc);
    d["SplitFinDesc"] = sizeof(SplitFinDesc);
    d["WgFinDesc"] = sizeof(WgFinDesc);
    d["ConvPoolDesc"] = sizeof(ConvPoolDesc);
    d["GChainDesc"] = sizeof(GChainDesc);
    d["RepBitsDesc"] = sizeof(RepBitsDesc);
    d["NbnDesc"] = sizeof(NbnDesc);
    d["AdamCtx"] = sizeof(AdamCtx);
    d["BinDesc"] = sizeof(BinDesc);
    return d;
}

PYBIND11_MODULE(serann_hip, m) {
    m.doc() = "SeRANN-AMD HIP/CDNA4 kernels (gfx950)";
    m.def("desc_sizes", &desc_sizes);
    m.def("src_hash", []() { return std::string(SERANN_SRC_HASH); });
    m.def("gemm3", &launch_gemm3, py::arg("mode"), py::arg("variant"), py::arg("descs"), py::arg("tiles"),
          py::arg("ntiles"), py::arg("stream"));
    m.def("transpose_weights", &launch_transpose_weights);
    m.def("adam", &launch_adam, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("pbf"), py::arg("step"),
          py::arg("lr_t"), py::arg("n"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("stream"),
          py::arg("mode") = 0);
    m.def("f32_to_bf16", &launch_f32_to_bf16);
    m.def("gather_batch", &launch_gather_batch);
    m.def("counter_add", &launch_counter_add);
    m.def("bn", &launch_bn);
    m.def("nbn", &launch_nbn);
    m.def("adam_scalars", &launch_adam_scalars);
    m.def("adam_update", &launch_adam_update, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("pbf"),
          py::arg("lr_t"), py::arg("n"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("skip"), py::arg("stream"),
          py::arg("mode") = 0, py::arg("org_off") = 0, py::arg("diverged") = 0, py::arg("norg") = 0);
    m.def("pool", &launch_pool);
    m.def("convpool", &launch_convpool);
    m.def("gchain", &launch_gchain);
    m.def("copy2d", &launch_copy2d);
    m.def("ew", &launch_ew);
    m.def("loss", &launch_loss);
    m.def("memset32", &launch_memset32);
    m.def("group_argmax", &launch_group_argmax);
    m.def("imcol", &launch_imcol);
    m.def("embed_gather", &launch_embed_gather);
    m.def("splitk_finalize", &launch_splitk_finalize);
    m.def("wgrad_finalize", &launch_wgrad_finalize);
    m.def("rep_bits", &launch_rep_bits);
    m.def("concrete_fwd", &launch_concrete_fwd, py::arg("logits"), py::arg("u"), py::arg("s"), py::arg("z"), py::arg("kl"),
          py::arg("B"), py::arg("G"), py::arg("A"), py::arg("t"), py::arg("tp"), py::arg("seed"), py::arg("offset"),
          py::arg("stream"), py::arg("zb") = 0);
    m.def("concrete_bwd", &launch_concrete_bwd, py::arg("s"), py::arg("z"), py::arg("gz"), py::arg("gkl"), py::arg("dlogits"),
          py::arg("B"), py::arg("G"), py::arg("A"), py::arg("t"), py::arg("tp"), py::arg("stream"), py::arg("bf16") = 0);
    m.def("cat_loglik_fwd", &launch_cat_loglik_fwd, py::arg("z"), py::arg("x"), py::arg("out"), py::arg("B"), py::arg("L"),
          py::arg("V"), py::arg("stream"), py::arg("bf16") = 0);
    m.def("cat_loglik_bwd", &launch_cat_loglik_bwd, py::arg("z"), py::arg("x"), py::arg("gout"), py::arg("dz"), py::arg("B"),
          py::arg("L"), py::arg("V"), py::arg("stream"), py::arg("bf16") = 0);
    m.def("onehot", &launch_onehot);
    m.def("bin", &launch_bin);
}
