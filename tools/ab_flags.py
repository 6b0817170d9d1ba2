"""A/B the C2 step and its zz^T kernel under snd_debug_set flags (plan-time choices).

    python tools/ab_flags.py --flags 0,4096
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from snd_vae_amd import _lib
    from snd_vae_amd.config import tscale
    from snd_vae_amd.parallel import init_from_env
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="0")
    ap.add_argument("--kernels", default="zzt_dense")
    ap.add_argument("--graphs", default="8", help="graphs per GPU, comma list")
    ap.add_argument("--config", default="", help="preset (C5, ...) instead of tscale(4096, 64)")
    ns = ap.parse_args()
    args = argparse.Namespace(steps=50, warmup=10, no_graph=False, dtype="bf16", no_tiles=False)
    info = init_from_env("nccl")
    for B in [int(x) for x in ns.graphs.split(",")]:
        for f in [int(x) for x in ns.flags.split(",")]:
            _lib.check(_lib.lib().snd_debug_set(f))
            from snd_vae_amd.config import PRESETS
            cfg = PRESETS[ns.config] if ns.config else tscale(4096, 64)
            v, ms, model, opt, db, host = bench.run_workload(cfg, B, args, info)
            kms = bench.kernel_timer(model, db.c_struct(), 20)
            ks = {k: round(kms(k), 5) for k in ns.kernels.split(",") if k}
            _lib.check(_lib.lib().snd_debug_set(0))
            print(f"B {B} flags {f}: step {ms:.4f} ms, {v:.1f} graphs/s, {ks}, "
                  f"cost {opt.loss_dict()['cost']:.6f}", flush=True)
            bench.del_models()


if __name__ == "__main__":
    main()
