"""One A/B measurement process: the C2 bench step (HIP-graph replay) and named plan
kernels timed with HIP events, for the library SND_LIB_PATH points at.

    SND_LIB_PATH=ab/x.so python tools/ab_run.py [--kernels zzt_dense,...] [--tag x]
Prints one JSON line.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="zzt_dense")
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--latent", type=int, default=64)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default=os.environ.get("SND_LIB_PATH", "default"))
    ap.add_argument("--config", default="", help="preset (C4, C5, ...) instead of --nodes/--latent")
    ap.add_argument("--adam-per-range", action="store_true",
                    help="A/B: one snd_adam_tf1 launch per unfused range instead of snd_adam_tf1_ranges")
    ap.add_argument("--debug", default="", help="comma list of snd_debug_set bits: each kernel is timed under each")
    ap.add_argument("--option", action="append", default=[],
                    help="plan option name=value (snd_plan_set_option), e.g. conc_decoder=1")
    ap.add_argument("--step-debug", type=int, default=0,
                    help="snd_debug_set bits for the captured step itself (host-side A/B switches)")
    args = ap.parse_args()
    import torch

    import bench
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    from snd_vae_amd.config import PRESETS
    if args.step_debug:
        _lib.lib().snd_debug_set(args.step_debug)
        args.tag += f" dbg{args.step_debug}"
    cfg = PRESETS[args.config] if args.config else tscale(args.nodes, args.latent)
    db = DeviceBatch(synthetic_batch(cfg, args.graphs, seed=1000))
    model = SGCNModelVAE(cfg, args.graphs, dtype="bf16")
    for o in args.option:
        k, v = o.split("=")
        args.tag += f" {k}={v}:{int(model.set_option(k, int(v)))}"
    opt = OptimizerVAE(model)
    if args.adam_per_range:
        def per_range(stream=None):
            for off, n in opt._adam_ranges:
                opt._adam(off, n, opt.grads[off:off + n], stream)
        opt.apply = per_range
        args.tag += " per-range"
    opt.step(db)
    opt.capture(db, warmup=2)
    for _ in range(10):
        opt.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        opt.replay()
    e1.record()
    e1.synchronize()
    out = {"tag": args.tag, "step_ms": round(e0.elapsed_time(e1) / args.steps, 5),
           "losses": {k: round(v, 6) for k, v in opt.loss_dict().items()}}
    km = bench.kernel_timer(model, db.c_struct(), args.reps)
    for d in [int(v) for v in args.debug.split(",") if v] or [None]:
        if d is not None:   # measurement library (-DSND_MEAS=1): phase-skip bits at launch time
            _lib.lib().snd_debug_set(d)
        sfx = "" if d is None else f"_dbg{d}"
        for k in [k for k in args.kernels.split(",") if k]:
            out[k + sfx + "_us"] = round(1000 * min(km(k) for _ in range(3)), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
