#!/usr/bin/env python
"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes (measurement tool).

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR [--key K --out profiles/traffic.json]
                                [--alg-bytes B]
Entries are stamped with the SHA-256 (16 hex digits) of the library the run loaded; bench.py only
reports an entry whose stamp matches the library it loads (a kernel change makes it stale).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (summed over the TCC instances).  On gfx950
FETCH_SIZE reports exactly half of the bytes of a wide coalesced streaming read
(MI355X_MICROARCH.md §HBM), so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for 16-B
streaming stores.  Prints the median over the kernel's dispatches and optionally merges
{key: bytes_per_launch} into the traffic JSON bench.py reads.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def per_dispatch(d, counter, kernel):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                key = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("kernel")
    ap.add_argument("--key")
    ap.add_argument("--out")
    ap.add_argument("--alg-bytes", type=float, default=None)
    ap.add_argument("--lib", default=None, help="library the profiled run loaded (default: in-tree)")
    ap.add_argument("--key-from", default=None,
                    help="take --key from config.traffic_key of this bench.py JSON output")
    a = ap.parse_args()
    if a.key_from:
        with open(a.key_from) as fh:
            line = [ln for ln in fh if ln.startswith("{")][-1]
        a.key = json.loads(line)["config"]["traffic_key"]
    f = per_dispatch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    w = per_dispatch(a.write_dir, "WRITE_SIZE", a.kernel)
    if not f or not w:
        raise SystemExit(f"no dispatches of {a.kernel!r} with counters (fetch {len(f)}, write {len(w)})")
    rd = 2 * statistics.median(f) * 1024
    wr = statistics.median(w) * 1024
    tot = rd + wr
    res = {"read_bytes": rd, "write_bytes": wr, "bytes": tot, "dispatches": [len(f), len(w)],
           "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count), write = WRITE_SIZE x 1024"}
    if a.alg_bytes:
        res["ratio_to_algorithmic"] = tot / a.alg_bytes
    print(json.dumps(res))
    if a.out and a.key:
        # entries are keyed by config/kernel/p/layout and stamped with the library they were
        # measured with: bench.py reports an entry only while the loaded library has that hash
        import hashlib
        lib = a.lib or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "non-iid-topology-simulator_amd", "niidmix", "libniidmix.so")
        with open(lib, "rb") as fh:
            res["lib_sha16"] = hashlib.sha256(fh.read()).hexdigest()[:16]
        data = {"entries": {}}
        if os.path.exists(a.out):
            with open(a.out) as fh:
                data = json.load(fh)
            data.setdefault("entries", {})
        data["entries"][a.key] = res
        with open(a.out, "w") as fh:
            json.dump(data, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
