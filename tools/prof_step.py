"""Run a few eager (non-graph) train steps for per-dispatch PMC profiling, or (--graph)
replays of the captured step for a kernel trace of the bench's own path.

    rocprofv3 --pmc SQ_WAVES ... -d gpurun_out/pmcX -o run --output-format csv -- \
        python tools/prof_step.py --steps 3
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--latent", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--config", default="", help="preset (C4, C5, ...) instead of --nodes/--latent")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step in a HIP graph and time REPLAYS (the bench's path; side-stream "
                         "concurrency as the bench runs it) instead of eager steps")
    ap.add_argument("--debug", type=int, default=0, help="snd_debug_set bits for the steps (A/B switches)")
    args = ap.parse_args()
    import torch
    from snd_vae_amd.config import PRESETS, tscale
    from snd_vae_amd.data import default_tile_rows, synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    if args.debug:
        from snd_vae_amd import _lib
        _lib.lib().snd_debug_set(args.debug)
    cfg = PRESETS[args.config] if args.config else tscale(args.nodes, args.latent)
    db = DeviceBatch(synthetic_batch(cfg, args.graphs, seed=1000), tile_rows=default_tile_rows(cfg.g_conv_hidden[1]))
    model = SGCNModelVAE(cfg, args.graphs, dtype=args.dtype)
    opt = OptimizerVAE(model)
    if args.graph:
        opt.capture(db)
        for _ in range(args.steps):
            opt.replay()
    else:
        for _ in range(args.steps):
            opt.step(db)
    torch.cuda.synchronize()
    print("ok", args.steps)


if __name__ == "__main__":
    main()
