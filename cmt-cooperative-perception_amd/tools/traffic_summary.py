"""HBM traffic per launch of the cross-attention kernel from the FETCH_SIZE /
WRITE_SIZE rocprofv3 passes of tools/profile_bench.sh, corrected as
MI355X_MICROARCH.md prescribes (gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads -> x2; WRITE_SIZE exact for 16-B stores).
Writes profiles/attn_pmc_summary.json.

    python cmt-cooperative-perception_amd/tools/traffic_summary.py gpurun_out/prof_r1 [--out profiles/attn_pmc_summary.json]
"""
import argparse
import glob
import json
import os
import sqlite3
import statistics


def per_kernel(db_path, counter):
    db = sqlite3.connect(db_path)
    rows = db.execute("select kernel_name, counter_name, value from counters_collection").fetchall()
    out = {}
    for k, c, v in rows:
        if c == counter:
            out.setdefault(k, []).append(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="profiles/attn_pmc_summary.json")
    ap.add_argument("--match", default="attn_pp_kernel")
    a = ap.parse_args()
    fdb = glob.glob(os.path.join(a.dir, "fetch", "**", "*.db"), recursive=True)[0]
    wdb = glob.glob(os.path.join(a.dir, "write", "**", "*.db"), recursive=True)[0]
    fetch = per_kernel(fdb, "FETCH_SIZE")
    write = per_kernel(wdb, "WRITE_SIZE")
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py (no graph); "
                     "FETCH_SIZE x2 (gfx950 wide-read correction), units KB -> bytes",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = statistics.median(fetch.get(k, [0])) * 1024 * 2
        w = statistics.median(write.get(k, [0])) * 1024
        res["kernels"][k] = {"fetch_bytes": f, "write_bytes": w, "launches": len(fetch.get(k, []))}
    attn = [v for k, v in res["kernels"].items() if a.match in k]
    if attn:
        res["hbm_bytes_per_launch"] = max(v["fetch_bytes"] + v["write_bytes"] for v in attn)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
