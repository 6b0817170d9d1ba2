"""MI355X-native SND-VAE training hot path (gfx950 HIP kernels behind a C ABI).

Package map:
  csrc/        HIP kernels + C ABI (libsndvae.so): CSR SpMM, MFMA GEMM/conv1d,
               fused zz^T + CE, reparam/KL, heads, TF1 Adam, train-step plan
  config.py    flags / presets (main.py:42-217)
  data.py      spatial-graph batches, CSR ingest (input_data.py, preprocessing.py)
  params.py    flat parameter layout + reference initialisers
  model.py     SGCNModelVAE (model.py / model_joint.py mirror)
  optimizer.py OptimizerVAE (optimizer.py mirror) + HIP-graph capture
  layers.py    functional op API (layers.py mirror)
  parallel.py  data parallelism (RCCL all-reduce)
  trainer.py   train loop (main.py:310-353 mirror)
"""
from .config import PRESETS, SNDConfig, tscale  # noqa: F401

__version__ = "0.1.0"
