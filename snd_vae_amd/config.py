"""Configuration for the SND-VAE training hot path.

Mirrors the flag block of the reference driver (`main.py:42-103`) and the
`synthetic2` dataset overrides (`main.py:173-217`), restricted to the fields the
hot path reads.  Named presets C1..C5 are the BASELINE.json configs.

Two decoder-input topologies exist (SURVEY.md §8 "Composed step"):

* ``tscale`` (C2/C3/C5): node-level latent.  The encoder heads
  (`model.py:113-115`) are applied per node row, so mu/logstd are [N, L] and
  the inner-product decoder input is J = z (L == node_h).
* ``tref`` (C1/C4): graph-level latent exactly as `model.py:113-115` +
  `model_joint.py:97` ('d_sg_lin1'): h = flat(G) W_h + b_h per graph,
  z [B, L], J = reshape(z W_p + b_p, [N, node_h]).

``encoder_coords`` appends the coordinates to the encoder input (SURVEY §8
decision iii): on for tscale and for C4 (whose flat(G) width 4096*67 is the
SURVEY §8a row a5 figure), off for C1, which keeps F_in = num_feature exactly
as `model.py:104`.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Tuple

# Keras BatchNormalization default epsilon (model.py:41, model_joint.py:25);
# frozen moving stats (mean 0, var 1) => y = gamma * x / sqrt(1 + eps) + beta.
BN_EPS = 1e-3
# lrelu leak (layers.py:112-113)
LRELU_LEAK = 0.2
# conv1d kernel size and SAME padding (main.py:199-206, model_joint.py:115,138)
CONV_K = 5


@dataclass(frozen=True)
class SNDConfig:
    n_nodes: int = 4096                 # N, nodes per spatial graph
    g_latent_size: int = 64             # L (main.py:191); == d for tscale
    topology: str = "tscale"            # "tscale" | "tref"
    num_feature: int = 1                # main.py:83
    spatial_dim: int = 2                # main.py:84
    g_conv_hidden: Tuple[int, int] = (64, 64)   # main.py:189 (widened)
    g_hidden_size: int = 64             # main.py:190
    node_h_size: int = 64               # main.py:209 (== latent for tscale)
    s_d_channel: Tuple[int, int, int] = (50, 20, 10)   # main.py:199
    n_d_channel: Tuple[int, int] = (50, 20)            # main.py:204 [:graph_deconv_layers]
    learning_rate: float = 0.0008       # main.py:211 (synthetic2)
    beta: float = 1.0                   # main.py:515 main(1, t)
    adam_beta1: float = 0.9             # tf.train.AdamOptimizer defaults
    adam_beta2: float = 0.999
    adam_eps: float = 1e-8
    mean_degree: float = 16.0           # synthetic RGG k-bar
    seed: int = 0
    weighted_bce: bool = False          # design decision (ii): off == reference
    pos_weight: float = 1.0
    norm: float = 1.0
    encoder_coords: bool = True         # X = [x_feat || S] (decision iii)
    # sgjoint: the spatial-graph encoder over sampling_num spanning trees per graph
    sampling_num: int = 10              # main.py:100
    sg_conv_hidden: Tuple[Tuple[int, int, int], ...] = ((20, 20, 20), (50, 50, 50))   # main.py:193

    @property
    def f_in(self) -> int:
        """Encoder input width (coordinates appended when encoder_coords; the
        spatial-graph encoder reads the coordinates through rel instead)."""
        if self.topology == "sgjoint":
            return self.num_feature
        if self.encoder_coords:
            return self.num_feature + self.spatial_dim
        return self.num_feature

    @property
    def latent(self) -> int:
        return self.g_latent_size

    @property
    def enc_width(self) -> int:
        """Width of G = BN_enc([BN(P1) || X]) (model.py:109-112); sgjoint: the last
        spatial-graph layer's width (model_joint.py:77-80)."""
        if self.topology == "sgjoint":
            return self.sg_conv_hidden[-1][2]
        return self.g_conv_hidden[1] + self.f_in

    def replace(self, **kw) -> "SNDConfig":
        return dataclasses.replace(self, **kw)


def tscale(n_nodes: int, latent: int, **kw) -> SNDConfig:
    """Node-latent topology with every width equal to d (SURVEY §8 config widths)."""
    return SNDConfig(n_nodes=n_nodes, g_latent_size=latent, topology="tscale",
                     g_conv_hidden=(latent, latent), g_hidden_size=latent,
                     node_h_size=latent, **kw)


def tref(n_nodes: int, node_h: int, g_hidden: int = 100, latent: int = 100,
         **kw) -> SNDConfig:
    """Graph-latent topology: g_hidden = L = 100 (main.py:190-191), node_h = d."""
    return SNDConfig(n_nodes=n_nodes, g_latent_size=latent, topology="tref",
                     g_conv_hidden=(node_h, node_h), g_hidden_size=g_hidden,
                     node_h_size=node_h, **kw)


def sgjoint(n_nodes: int, node_h: int, g_hidden: int = 100, latent: int = 100,
            sampling_num: int = 10, sg_conv_hidden=((20, 20, 20), (50, 50, 50)), **kw) -> SNDConfig:
    """The SND-VAE spatial-graph encoder (model_joint.py:72-85, model.py:134-151):
    two SpatialGraphConvolution layers over sampling_num spanning trees per graph,
    flat heads per tree copy (sg_hidden_size = g_hidden, sg_latent_size = latent,
    main.py:194-195), z averaged over the copies after d_sg_lin1 (model.py:177,180),
    then the graph-latent decoders.  Synthetic2 widths by default (main.py:173-217)."""
    kw.setdefault("encoder_coords", False)   # coordinates enter through rel
    return SNDConfig(n_nodes=n_nodes, g_latent_size=latent, topology="sgjoint",
                     g_conv_hidden=(node_h, node_h), g_hidden_size=g_hidden, node_h_size=node_h,
                     sampling_num=sampling_num,
                     sg_conv_hidden=tuple(tuple(int(v) for v in h) for h in sg_conv_hidden), **kw)


PRESETS = {
    # C1: N=200 d=16, reference CPU plumbing.  tref as in model.py:104.
    "C1": tref(200, 16, mean_degree=8.0, encoder_coords=False),
    # C1 in the node-latent topology (used for GPU parity at small N).
    "C1s": tscale(200, 16, mean_degree=8.0),
    # C2: N=4096 d=64 bf16 on 1 GPU -- the bench workload.
    "C2": tscale(4096, 64),
    # C3: C2 graphs data-parallel over 8 GPUs.
    "C3": tscale(4096, 64),
    # C4: model_joint structure + coordinate decoders on the graph latent, N=4096 d=64.
    "C4": tref(4096, 64),
    # C5: N=16384 d=128 inner-product decoder stress.
    "C5": tscale(16384, 128),
    # The reference's own scale for the spatial-graph encoder: synthetic2, N=25,
    # 10 spanning trees per graph (main.py:100,173-217).
    "SG25": sgjoint(25, 16, mean_degree=4.0),
}
