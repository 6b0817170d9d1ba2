#!/usr/bin/env python3
"""Write tests/parity_bars.json from recorded GPU parity errors.

usage: python tools/make_bars.py [errors.jsonl ...]   (default gpurun_out/parity_errors.jsonl)

For every bf16 test case (the record's "test" field) and every quantity, the bar is
FACTOR[kind] x the largest error recorded for it (over steps and files), rounded up to
two significant digits, at least FLOOR[kind] (tests/parity_bars.py).  Round-5 records
(keys loss_rel / grad_err / m_err / v_err, test names without the "/dtype" suffix) are
read too.  Existing table entries for cases the inputs do not mention are kept.
"""
import collections
import datetime
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import parity_bars as PB  # noqa: E402

OLD = {"loss_rel": "loss", "grad_err": "grad", "m_err": "m", "v_err": "v"}
OLD_CASE = {"c2_bench_batch_steps": "c2_bench_steps", "c4_bench_batch": None}


def case_of(r):
    t = r["test"]
    if "/" in t:
        return t
    base = OLD_CASE.get(t, t)
    if base is None:   # c4: the schedule from the lr
        base = "c4_bench_lr1e-6" if r.get("lr") == 1e-6 else "c4_bench_reflr"
    return f"{base}/{r['dtype']}"


def main(paths):
    worst = collections.defaultdict(lambda: collections.defaultdict(float))
    sources = []
    for path in paths:
        sources.append(os.path.relpath(path, ROOT))
        for line in open(path):
            r = json.loads(line)
            if r.get("dtype") != "bf16":
                continue
            case = case_of(r)
            for key, val in r.items():
                kind = OLD.get(key, key)
                if kind not in PB.FACTOR or not isinstance(val, dict):
                    continue
                for q, e in val.items():
                    if isinstance(e, (int, float)):
                        k = f"{kind}:{q}"
                        worst[case][k] = max(worst[case][k], float(e))
    table = {}
    if os.path.exists(PB.TABLE):
        table = json.load(open(PB.TABLE)).get("bars", {})
    for case, qs in worst.items():
        table[case] = {k: max(PB.FLOOR[k.split(":")[0]], PB.round_up2(PB.FACTOR[k.split(":")[0]] * e))
                       for k, e in sorted(qs.items())}
    out = {"note": "bf16 parity bars: FACTOR x the largest recorded error per test case and "
                   "quantity (tests/parity_bars.py; written by tools/make_bars.py)",
           "factor": PB.FACTOR, "floor": PB.FLOOR,
           "sources": sources, "written": datetime.date.today().isoformat(),
           "bars": dict(sorted(table.items()))}
    with open(PB.TABLE, "w") as f:
        json.dump(out, f, indent=1, sort_keys=False)
        f.write("\n")
    print(f"{PB.TABLE}: {len(table)} cases, {sum(len(v) for v in table.values())} bars")


if __name__ == "__main__":
    main(sys.argv[1:] or [os.path.join(ROOT, "gpurun_out", "parity_errors.jsonl")])
