#!/usr/bin/env python3
"""Per-launch SQ counters of scripts/newton_ceiling.hip under rocprofv3 (scripts/newton_ceiling.sh), grouped by the
probe's waves per SIMD: the probe launches k_ceiling 6 times per W (one warm-up, five timed) for W = 1, 2, 4, 6, 8,
in that order, so dispatch k belongs to W index k // 6.  One JSON line per W: the counters' means over its launches
and the kernel-trace mean duration.

usage: python scripts/newton_ceiling_pmc.py gpurun_out/newton_ceiling
"""
import glob
import json
import sqlite3
import sys
from collections import defaultdict

WS = (1, 2, 4, 6, 8)
PER_W = 6


def rows(db, sql):
    c = sqlite3.connect(db)
    try:
        return list(c.execute(sql))
    except sqlite3.OperationalError as e:
        print(f"{db}: {e}", file=sys.stderr)
        return []


def cols(db, table):
    return [r[1] for r in rows(db, f"pragma table_info({table})")]


def main():
    d = sys.argv[1]
    out = defaultdict(dict)
    for db in sorted(glob.glob(f"{d}/sq1/**/*.db", recursive=True)):
        cc = cols(db, "counters_collection")
        key = "dispatch_id" if "dispatch_id" in cc else ("correlation_id" if "correlation_id" in cc else "rowid")
        r = rows(db, f"select {key}, kernel_name, counter_name, value from counters_collection")
        ids = sorted({x[0] for x in r if "k_ceiling" in x[1]})
        rank = {i: k for k, i in enumerate(ids)}
        acc = defaultdict(lambda: defaultdict(list))
        for i, name, cn, v in r:
            if "k_ceiling" in name:
                acc[WS[min(rank[i] // PER_W, len(WS) - 1)]][cn].append(v)
        for w, cs in acc.items():
            out[w].update({cn: sum(v) / len(v) for cn, v in cs.items()})
            out[w]["launches"] = max(len(v) for v in cs.values())
    for db in sorted(glob.glob(f"{d}/trace/**/*.db", recursive=True)):
        cc = cols(db, "kernels")
        if "start" in cc and "end" in cc:
            r = rows(db, "select name, start, end from kernels order by start")
            durs = [(e - s) / 1e6 for n, s, e in r if "k_ceiling" in n]
            for k, w in enumerate(WS):
                part = durs[k * PER_W + 1:(k + 1) * PER_W]
                if part:
                    out[w]["trace_ms_mean_timed"] = sum(part) / len(part)
        else:
            print(f"{db}: kernels view has columns {cc}", file=sys.stderr)
    for w in WS:
        if w in out:
            print(json.dumps({"waves_per_simd": w, **out[w]}))


if __name__ == "__main__":
    main()
