"""Time the bf16 decoder kernels one at a time (HIP events on the launch stream),
optionally with measurement-only phase-skip flags (snd_debug_set).

    python tools/ab_fast.py [--flags 0,1,2,4,8]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

NAMES = ["conv1 fwd", "conv2 fwd", "conv3 fwd", "heads", "conv3 bwd-data", "conv3 wgrad",
         "conv2 bwd-data", "conv2s wgrad", "conv2n wgrad", "conv1 bwd-data", "conv1 wgrad"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="0")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--graphs", type=int, default=8)
    ap.add_argument("--keys", default="", help="snd_plan_launch keys, comma list (default: pack + dec:0..10)")
    args = ap.parse_args()
    import torch
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.data import synthetic_batch
    from snd_vae_amd.model import DeviceBatch, SGCNModelVAE
    from snd_vae_amd.optimizer import OptimizerVAE
    cfg = tscale(4096, 64)
    db = DeviceBatch(synthetic_batch(cfg, args.graphs, seed=1000))
    model = SGCNModelVAE(cfg, args.graphs, dtype="bf16")
    opt = OptimizerVAE(model)
    opt.step(db)
    torch.cuda.synchronize()
    bc = db.c_struct()
    L = _lib.lib()
    st = _lib.stream_ptr()
    flags = [int(f, 0) for f in args.flags.split(",")]
    keys = ["pack"] + [f"dec:{k}" for k in range(len(NAMES))]
    labels = ["pack"] + NAMES
    if args.keys:
        keys = args.keys.split(",")
        labels = keys
    print("kernel".ljust(18) + "".join(f"flags={f:<4d}".rjust(12) for f in flags))
    for key, lab in zip(keys, labels):
        row = []
        for f in flags:
            _lib.check(L.snd_debug_set(f))
            # capture reps launches in one HIP graph: times the GPU, not the host
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(), key.encode(),
                                             _lib.stream_ptr(s)))
                with torch.cuda.graph(g, stream=s):
                    for _ in range(args.reps):
                        _lib.check(L.snd_plan_launch(model.plan, bc, model.workspace.data_ptr(),
                                                     key.encode(), _lib.stream_ptr(s)))
            torch.cuda.current_stream().wait_stream(s)
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            row.append(e0.elapsed_time(e1) * 1e3 / (5 * args.reps))
        _lib.check(L.snd_debug_set(0))
        print(lab.ljust(18) + "".join(f"{v:12.2f}" for v in row))


if __name__ == "__main__":
    main()
