"""HBM bytes per launch of each render kernel kind from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

Usage: pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON WORKLOAD [FRAMES]

FRAMES: frames of WORKLOAD the passes ran (default 1); bench.py turns the bytes into bytes per sample
(launches x bytes per launch / (frames x samples per frame)) and uses them for any frame size and spp of the
same scene, depth and build.

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): both counters are in KiB; on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced read, so it is doubled; WRITE_SIZE is taken as is. bench.py reads OUT_JSON
(profiles/r1/pmc_traffic_c2.json) into roofline.traffic when its workload matches the bench's.
"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def source_id():
    """The build the counters were collected on (bench.py uses the file only for that build)."""
    import __graft_entry__
    return __graft_entry__.load_package().source_id()

KINDS = {"pt::wf_bounce<": "bounce", "pt::wf_march<": "march", "pt::wf_walk<": "walk", "pt::render_tiles": "megakernel"}


def kind_of(name):
    name = name.replace("void ", "")
    for prefix, kind in KINDS.items():
        if name.startswith(prefix):
            return kind
    return None


def collect(d, counter):
    tot = collections.defaultdict(float)
    ids = collections.defaultdict(set)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = kind_of(row["Kernel_Name"])
            if k is None or row["Counter_Name"] != counter:
                continue
            tot[k] += float(row["Counter_Value"]) * 1024.0
            ids[k].add(row.get("Dispatch_Id"))
    return tot, {k: len(v) for k, v in ids.items()}


def main():
    fetch_dir, write_dir, out, workload = sys.argv[1:5]
    frames = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    fetch, nf = collect(fetch_dir, "FETCH_SIZE")
    write, nw = collect(write_dir, "WRITE_SIZE")
    rec = {"workload": workload, "source_id": source_id(), "unit": "bytes per launch", "frames": frames,
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
           "kinds": {}}
    for k in sorted(set(fetch) & set(write)):
        rd = fetch[k] * 2.0 / nf[k]
        wr = write[k] / nw[k]
        rec["kinds"][k] = {"launches": nf[k], "read": rd, "write": wr, "traffic": rd + wr}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
