"""Summaries of rocprofv3 sqlite outputs (*_results.db): per-kernel time
(--kernel-trace) and per-kernel PMC counter totals (--pmc passes).

  python tools/rocpd_summary.py trace DB          -> kernel stats table
  python tools/rocpd_summary.py pmc DB [DB ...]   -> counters per kernel
"""
import sqlite3
import sys
from collections import defaultdict


def short(name):
    import re
    m = re.search(r"k_[a-z_]+(?:<[^>]*>)?", name)
    n = m.group(0) if m else name[:60]
    t = re.search(r"ILb(\d)E(?:Lb(\d)E)?", name)
    if t:
        n += "<" + ",".join(x for x in t.groups() if x is not None) + ">"
    return n


def trace(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, end - start from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0, 0.0, 1e30])
    for name, dur in rows:
        a = agg[short(name)]
        a[0] += 1
        a[1] += dur
        a[2] = max(a[2], dur)
        a[3] = min(a[3], dur)
    tot = sum(a[1] for a in agg.values())
    print(f"{'kernel':40s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>10s} {'min_us':>9s} {'max_us':>10s} {'pct':>6s}")
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:40s} {a[0]:7d} {a[1] / 1e6:10.2f} {a[1] / a[0] / 1e3:10.2f} {a[3] / 1e3:9.2f} {a[2] / 1e3:10.2f} "
              f"{100 * a[1] / tot:6.2f}")


def pmc(dbs, as_json=None):
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for db in dbs:
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
        name_col = "kernel_name" if "kernel_name" in cols else [x for x in cols if "kernel" in x and "name" in x][0]
        cn_col = "counter_name" if "counter_name" in cols else [x for x in cols if "counter" in x and "name" in x][0]
        val_col = [x for x in ("counter_value", "value") if x in cols][0]
        q = f"select {name_col}, {cn_col}, {val_col}, dispatch_id from counters_collection"
        for kname, cname, val, did in c.execute(q):
            agg[short(kname)][cname] += val
            disp[short(kname)].add(did)
    if as_json:
        import json
        out = {k: dict(d, dispatches=len(disp[k])) for k, d in agg.items()}
        with open(as_json, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
    for k, d in sorted(agg.items()):
        print(f"{k}  (dispatches: {len(disp[k])})")
        for cn, v in sorted(d.items()):
            print(f"   {cn:32s} {v:18.4g}")


if __name__ == "__main__":
    if sys.argv[1] == "trace":
        trace(sys.argv[2])
    elif sys.argv[1] == "pmcjson":
        pmc(sys.argv[3:], as_json=sys.argv[2])
    else:
        pmc(sys.argv[2:])
