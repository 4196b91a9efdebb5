"""Summarise a rocprofv3 counter database (rocpd SQLite): per kernel name the
dispatch count, mean duration and the mean of every collected counter.

    python dev/pmc_summary.py gpurun_out/<dir>/run_results.db [--match attn]
"""
import argparse
import collections
import json
import sqlite3


def summarise(path, match=""):
    db = sqlite3.connect(path)
    rows = db.execute("select dispatch_id, kernel_name, counter_name, value, start, end from counters_collection")
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(dict)
    for did, kname, cname, val, st, en in rows:
        if match and match not in kname:
            continue
        per[kname][cname].append(val)
        durs[kname][did] = en - st
    out = {}
    for k, cs in per.items():
        d = list(durs[k].values())
        out[k] = {"dispatches": len(d), "mean_duration_us": sum(d) / len(d) / 1e3,
                  **{c: sum(v) / len(v) for c, v in sorted(cs.items())}}
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    print(json.dumps(summarise(a.db, a.match), indent=1))
