"""SeRANN-AMD: an MI355X-native framework for evolutionary experiments with
Self-Replicating Artificial Neural Networks.

Capability parity target: yoavram-lab/Self-Replicating-Artificial-Neural-Networks
(see SURVEY.md).  Layout:

* ``serann.genome``     tokenizer, genome interpreter (source -> layer IR),
                        synthetic SeRANN generator, genetic codecs
* ``serann.models``     torch oracle organism, ribosomal autoencoder model
* ``serann.engine``     population training engines (torch oracle, HIP grouped)
* ``serann.ops``        HIP/CDNA4 kernels (grouped MFMA GEMM/conv, BN, Adam, ...)
* ``serann.parallel``   SPMD over torch.distributed (RCCL on GPU, gloo on CPU)
* ``serann.experiment`` generation loop (fertility, selection, proofreading)
* ``serann.evaluation`` retrospective fertility / mutation-rate evaluation
* ``serann.riboae``     ribosomal autoencoder trainer
* ``serann.utils``      SQLite results DB, population statistics, Levenshtein
* ``serann.analysis``   results loaders, Muller-plot preparation
"""

__version__ = "0.1.0"
