"""HBM traffic per launch of the cross-attention kernel (core + its split
combine) from the FETCH_SIZE / WRITE_SIZE rocprofv3 passes of
dev/gpu_check.sh (prof), corrected as MI355X_MICROARCH.md prescribes
(gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads ->
x2; WRITE_SIZE exact for 16-B stores).  Writes
profiles/<tag>_<workload>_attn_pmc_summary.json, which bench.py's
load_traffic() keys on (workload, nk).

    python dev/traffic_summary.py gpurun_out/<tag>/prof \
        --tag r2a --workload fusion --nk 56400 [--match attn_pb_kernel --match 'attn_combine_kernel<8>']
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
    ap.add_argument("--tag", required=True)
    ap.add_argument("--workload", required=True)
    ap.add_argument("--nk", type=int, required=True)
    ap.add_argument("--match", action="append", default=None,
                    help="kernel-name substrings whose per-launch medians add up to one cross-attention launch")
    ap.add_argument("--outdir", default="profiles")
    a = ap.parse_args()
    match = a.match
    fdb = glob.glob(os.path.join(a.dir, "fetch", "**", "*.db"), recursive=True)[0]
    wdb = glob.glob(os.path.join(a.dir, "write", "**", "*.db"), recursive=True)[0]
    fetch = per_kernel(fdb, "FETCH_SIZE")
    write = per_kernel(wdb, "WRITE_SIZE")
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py (no graph); "
                     "FETCH_SIZE x2 (gfx950 wide-read correction), units KB -> bytes; per-launch medians",
           "workload": a.workload, "nk": a.nk, "match": match, "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = statistics.median(fetch.get(k, [0])) * 1024 * 2
        w = statistics.median(write.get(k, [0])) * 1024
        res["kernels"][k] = {"fetch_bytes": f, "write_bytes": w, "launches": len(fetch.get(k, []))}
    if match is None:
        # the bounded bf16 core (attn_pb2_kernel paired-tile / attn_pb_kernel) or the ping-pong core
        # (attn_pp_kernel), + its split combine
        core = next((c for c in ("attn_pb2_kernel", "attn_pb_kernel")
                     if any(c in k for k in res["kernels"])), "attn_pp_kernel")
        match = res["match"] = [core, "attn_combine_kernel<8>"]
    parts = {}
    for m in match:
        hits = [(k, v) for k, v in res["kernels"].items() if m in k]
        if not hits:
            raise SystemExit(f"no kernel matches {m!r}")
        k, v = max(hits, key=lambda kv: kv[1]["fetch_bytes"] + kv[1]["write_bytes"])
        parts[k] = v["fetch_bytes"] + v["write_bytes"]
    res["parts"] = parts
    res["hbm_bytes_per_launch"] = sum(parts.values())
    out = os.path.join(a.outdir, f"{a.tag}_{a.workload}_attn_pmc_summary.json")
    os.makedirs(a.outdir, exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(out, json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))


if __name__ == "__main__":
    main()
