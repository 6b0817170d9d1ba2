"""Time the C2 train step (HIP-graph replay, HIP events on the replay stream) of the
package under --root, so several source trees can be A/B'd in alternating processes
on one box.  Prints one JSON line.

    python tools/step_time.py --root _bisect/7654dd2 --graphs 8 --steps 200
"""
import argparse
import json
import os
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--nodes", type=int, default=4096)
    ap.add_argument("--latent", type=int, default=64)
    ap.add_argument("--config", default="")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--eager", type=int, default=0, help="run N eager steps (for rocprof) and exit")
    ap.add_argument("--option", action="append", default=[], help="plan option name=value")
    ap.add_argument("--tag", default="")
    ap.add_argument("--debug", type=int, default=0, help="snd_debug_set bits before the plan is built (A/B)")
    args = ap.parse_args()
    root = os.path.abspath(args.root)
    sys.path.insert(0, root)
    import torch
    from snd_vae_amd.config import PRESETS, tscale
    from snd_vae_amd.data import default_tile_rows, synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    import snd_vae_amd
    assert os.path.dirname(os.path.abspath(snd_vae_amd.__file__)).startswith(root), snd_vae_amd.__file__
    if args.debug:
        from snd_vae_amd import _lib
        _lib.lib().snd_debug_set(args.debug)
    cfg = PRESETS[args.config] if args.config else tscale(args.nodes, args.latent)
    host = synthetic_batch(cfg, args.graphs, seed=1000)
    db = DeviceBatch(host, tile_rows=default_tile_rows(cfg.g_conv_hidden[1]))
    model = SGCNModelVAE(cfg, args.graphs, dtype=args.dtype)
    for o in args.option:
        k, v = o.split("=")
        model.set_option(k, int(v))
    opt = OptimizerVAE(model)
    opt.step(db)
    torch.cuda.synchronize()
    if args.eager:
        for _ in range(args.eager):
            opt.step(db)
        torch.cuda.synchronize()
        print(json.dumps({"tag": args.tag or os.path.basename(root), "eager_steps": args.eager,
                          "losses": {k: round(v, 6) for k, v in opt.loss_dict().items()}}))
        return
    opt.capture(db, warmup=2)
    for _ in range(20):
        opt.replay()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    for e0, e1 in ev:
        e0.record()
        opt.replay()
        e1.record()
    torch.cuda.synchronize()
    per = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    med = per[len(per) // 2]
    print(json.dumps({"tag": args.tag or os.path.basename(root), "graphs": args.graphs,
                      "ms_median": round(med, 5), "ms_min": round(per[0], 5),
                      "ms_p90": round(per[int(0.9 * len(per))], 5),
                      "losses": {k: round(v, 6) for k, v in opt.loss_dict().items()}}))


if __name__ == "__main__":
    main()
