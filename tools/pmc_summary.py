#!/usr/bin/env python3
"""Average each PMC counter per dispatch, per kernel, over a rocprofv3
counter_collection.csv (the last dispatches of every kernel: steady state).

With --json OUT, merge {kernel: {counter: value}} into OUT; FETCH_SIZE and
WRITE_SIZE (KB) also give hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024, the
gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of
wide coalesced reads)."""
import collections
import csv
import json
import os
import sys


def summarize(path, last=3):
    rows = list(csv.DictReader(open(path)))
    by = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("gw::", "")
        by[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    out = {}
    for k, cs in by.items():
        vals = {}
        for c, lst in cs.items():
            per = collections.defaultdict(float)     # sum over per-XCD rows of one dispatch
            for d, v in lst:
                per[d] += v
            ds = sorted(per)[-last:]
            vals[c] = sum(per[d] for d in ds) / len(ds)
        out[k] = vals
    return out


def finalize(argv):
    """Stamp a merged pass with the kernel-source hash bench.py checks and the
    config it was taken on: {"src_hash", "config", "kernels": {...}}."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    src = argv[argv.index("--finalize") + 1]
    cfg = int(argv[argv.index("--config") + 1])
    out = argv[argv.index("--out") + 1]
    kern = json.load(open(src))
    json.dump({"src_hash": bench.src_hash(), "config": cfg,
               "how": "rocprofv3 --pmc, one counter group per run (tools/gpu/pmc.sh), last 3 dispatches "
                      "averaged; hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KB -> B; gfx950 correction of "
                      "MI355X_MICROARCH.md)",
               "kernels": kern}, open(out, "w"), indent=1, sort_keys=True)
    print("wrote", out)


def main(argv):
    if "--finalize" in argv:
        return finalize(argv)
    path = argv[1]
    js = argv[argv.index("--json") + 1] if "--json" in argv else None
    out = summarize(path)
    for k, vals in sorted(out.items(), key=lambda kv: -max(kv[1].values()))[:14]:
        print(f"{k[:40]:40s} " + " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
    if js:
        cur = json.load(open(js)) if os.path.exists(js) else {}
        for k, vals in out.items():
            d = cur.setdefault(k, {})
            d.update(vals)
            if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
                d["hbm_bytes"] = 2 * d["FETCH_SIZE"] * 1024 + d["WRITE_SIZE"] * 1024
        json.dump(cur, open(js, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv)
