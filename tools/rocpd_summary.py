"""Summaries of rocprofv3 sqlite outputs (*_results.db): per-kernel time
(--kernel-trace) and per-kernel PMC counter totals (--pmc passes).

  python tools/rocpd_summary.py trace DB          -> kernel stats table
  python tools/rocpd_summary.py pmc DB [DB ...]   -> counters per kernel
  python tools/rocpd_summary.py gaps DB [JSON]    -> per stream: the idle time between one
                                                     kernel's end and the next one's start
"""
import sqlite3
import sys
from collections import defaultdict


def short(name):
    import re
    m = re.search(r"k_[a-z_]+(?:<[^>]*>)?", name)
    n = m.group(0) if m else name[:60]
    t = re.search(r"I((?:L[bi]\d+E)+)", name)
    if t:
        n += "<" + ",".join(re.findall(r"L[bi](\d+)E", t.group(1))) + ">"
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


def gaps(db, as_json=None):
    """Per stream (queue when the trace has no stream id), consecutive dispatches: the gap
    from one kernel's end to the next's start, split at 20 us (launch / dependency gaps vs
    host round trips), and per kernel pair."""
    import json
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    sid = [x for x in ("stream_id", "queue_id") if x in cols]
    key = sid[0] if sid else None
    rows = c.execute(f"select name, start, end{', ' + key if key else ''} from kernels order by start").fetchall()
    by = defaultdict(list)
    for r in rows:
        by[r[3] if key else 0].append((short(r[0]), r[1], r[2]))
    out = {"columns": cols, "group_by": key, "streams": {}}
    for s_, ks in by.items():
        g = [(ks[i - 1][0] + "->" + ks[i][0], (ks[i][1] - ks[i - 1][2]) / 1e3) for i in range(1, len(ks))]
        short_g = [x for _, x in g if x < 20.0]
        pairs = defaultdict(list)
        for pn, x in g:
            if x < 20.0:
                pairs[pn].append(x)
        srt = sorted(short_g)
        out["streams"][str(s_)] = {
            "kernels": len(ks), "gaps_under_20us": len(short_g),
            "median_us": round(srt[len(srt) // 2], 2) if srt else None,
            "mean_us": round(sum(srt) / len(srt), 2) if srt else None,
            "gaps_over_20us": sum(1 for _, x in g if x >= 20.0),
            "over_20us_total_ms": round(sum(x for _, x in g if x >= 20.0) / 1e3, 3),
            "pairs": {k: {"n": len(v), "median_us": round(sorted(v)[len(v) // 2], 2)} for k, v in pairs.items() if len(v) >= 4}}
    txt = json.dumps(out, indent=1)
    print(txt)
    if as_json:
        with open(as_json, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    if sys.argv[1] == "gaps":
        gaps(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
        sys.exit(0)
    if sys.argv[1] == "trace":
        trace(sys.argv[2])
    elif sys.argv[1] == "pmcjson":
        pmc(sys.argv[3:], as_json=sys.argv[2])
    else:
        pmc(sys.argv[2:])
