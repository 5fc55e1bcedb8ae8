"""Writes profiles/traffic.json's `<config>_1lane` entry from a tools/profile_roofline.sh
run: FETCH_SIZE / WRITE_SIZE of the non-stats (<false>) dispatches, which are the two
1-lane renders of `bench.py --roofline-only`, per dispatch. FETCH KB x 1024 x 2 (the
gfx950 FETCH_SIZE correction of /opt/skills/guides/MI355X_MICROARCH.md), WRITE KB x 1024.

  python tools/update_traffic.py ROOF_DIR [--config cfg2] [--build COMMIT] [--commit-dir profiles/NAME]

The per-pass summaries and PMC tables are copied to the committed directory (default
profiles/<basename of ROOF_DIR>), whose path the entry records.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, counter, scale):
    d = json.load(open(path))
    out = {}
    for k in ("k_trace", "k_step", "k_tail"):
        # every non-stats instantiation (<false> or <false, ...>)
        rs = [r for name, r in d.items() if name == f"{k}<false>" or name.startswith(f"{k}<false,")]
        n = sum(r.get("dispatches", 0) for r in rs)
        if n:
            out[k] = int(round(sum(r[counter] for r in rs) * 1024 * scale / n))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("roof_dir")
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--build", default="")
    ap.add_argument("--commit-dir", default=None)
    args = ap.parse_args()
    dest = args.commit_dir or os.path.join(REPO, "profiles", os.path.basename(os.path.normpath(args.roof_dir)))
    os.makedirs(dest, exist_ok=True)
    for f in glob.glob(os.path.join(args.roof_dir, "*.json")) + glob.glob(os.path.join(args.roof_dir, "*.summary.txt")):
        if os.path.abspath(os.path.dirname(f)) != os.path.abspath(dest):
            shutil.copy(f, dest)
    fetch = per_launch(os.path.join(args.roof_dir, "pmc_fetch.json"), "FETCH_SIZE", 2)
    write = per_launch(os.path.join(args.roof_dir, "pmc_write.json"), "WRITE_SIZE", 1)
    p = os.path.join(REPO, "profiles", "traffic.json")
    t = json.load(open(p)) if os.path.exists(p) else {}
    rel = os.path.relpath(dest, REPO)
    t[f"{args.config}_1lane"] = {
        "bytes_per_launch": fetch["k_trace"],
        "per_class_bytes_per_launch": fetch,
        "per_class_write_bytes_per_launch": write,
        "source": f"{rel}/pmc_fetch.json (FETCH_SIZE) and pmc_write.json (WRITE_SIZE): rocprofv3 --pmc over "
                  f"`bench.py --roofline-only --no-cpu-baseline --config {args.config}` (tools/profile_roofline.sh; "
                  "the <false> dispatches are the two 1-lane renders); FETCH KB x1024 x2 (gfx950 correction, "
                  "MI355X_MICROARCH.md), WRITE KB x1024, / dispatches" + (f"; build of commit {args.build}" if args.build else ""),
        "profile": f"{rel}/pmc_fetch.json",
        "build": args.build or None,
        "round": 5,
    }
    json.dump(t, open(p, "w"), indent=1)
    print(json.dumps(t[f"{args.config}_1lane"]))


if __name__ == "__main__":
    main()
