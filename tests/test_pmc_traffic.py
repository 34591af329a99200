"""scripts/pmc_traffic.py: per-launch HBM bytes from rocprofv3 --pmc counter CSVs (the source of bench.py's
roofline.traffic), checked on a synthetic two-pass CSV, and the committed C2 file's shape."""
import csv
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _pass(d, counter, rows):
    d.mkdir(parents=True)
    with open(d / "p_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (name, kib) in enumerate(rows):
            w.writerow({"Dispatch_Id": i, "Kernel_Name": name, "Counter_Name": counter, "Counter_Value": kib})


def test_pmc_traffic_corrections(tmp_path):
    b = "void pt::wf_bounce<4, false, 3, false, 0, false>(pt::dev::Scene)"
    m = "void pt::wf_march<false, 0>(pt::dev::Scene)"
    _pass(tmp_path / "f", "FETCH_SIZE", [(b, 100.0), (b, 300.0), (m, 10.0), ("pt::cp_scan(unsigned int*)", 5.0)])
    _pass(tmp_path / "w", "WRITE_SIZE", [(b, 50.0), (b, 50.0), (m, 4.0)])
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, str(ROOT / "scripts" / "pmc_traffic.py"), str(tmp_path / "f"),
                    str(tmp_path / "w"), str(out), "wl"], check=True, capture_output=True)
    rec = json.loads(out.read_text())
    assert rec["workload"] == "wl"
    bo = rec["kinds"]["bounce"]
    assert bo["launches"] == 2
    assert bo["read"] == 200.0 * 1024 * 2          # mean KiB per launch, x1024, x2 gfx950 FETCH_SIZE correction
    assert bo["write"] == 50.0 * 1024
    assert bo["traffic"] == bo["read"] + bo["write"]
    assert rec["kinds"]["march"]["traffic"] == (10.0 * 2 + 4.0) * 1024
    assert "cp_scan" not in json.dumps(rec["kinds"])


def test_committed_c2_traffic_matches_bench_workload():
    rec = json.loads((ROOT / "profiles" / "r1" / "pmc_traffic_c2.json").read_text())
    # bench.py's default config.workload string; the file is used only when they are equal
    assert rec["workload"] == "cornell_box.json 1920x1080 256spp depth 8"
    for kind in ("bounce", "march"):
        k = rec["kinds"][kind]
        assert k["launches"] > 0 and k["traffic"] > 0


def test_pmc_flops_lane_scaling(tmp_path):
    """scripts/pmc_flops.py: wave-instruction counts x mean active lanes / samples."""
    d = tmp_path / "sq"
    d.mkdir()
    b = "void pt::wf_bounce<4, false, 3, false, 0, false>(pt::dev::Scene)"
    rows = [("SQ_INSTS_VALU_ADD_F64", 100.0), ("SQ_INSTS_VALU_MUL_F64", 50.0), ("SQ_INSTS_VALU_FMA_F64", 10.0),
            ("SQ_INSTS_VALU_TRANS_F64", 2.0), ("SQ_THREAD_CYCLES_VALU", 3200.0), ("SQ_ACTIVE_INST_VALU", 100.0),
            ("SQ_INSTS_VALU", 400.0)]
    with open(d / "p_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for name, v in rows:
            w.writerow({"Dispatch_Id": 0, "Kernel_Name": b, "Counter_Name": name, "Counter_Value": v})
    out = tmp_path / "f.json"
    subprocess.run([sys.executable, str(ROOT / "scripts" / "pmc_flops.py"), str(d), "2", "10", str(out), "wl"],
                   check=True, capture_output=True)
    k = json.loads(out.read_text())["kinds"]["bounce"]
    assert k["mean_active_lanes"] == 32.0
    # per frame 50 ADD, 25 MUL wave instructions x 32 lanes / 10 samples
    assert k["algorithmic_flops_per_sample"] == (50 + 25) * 32 / 10
    assert k["executed_flops_per_sample"] == (50 + 25 + 2 * 5 + 1) * 32 / 10


def test_committed_c2_flops_match_bench_workload():
    rec = json.loads((ROOT / "profiles" / "r2" / "pmc_flops_c2.json").read_text())
    assert rec["workload"] == "cornell_box.json 1920x1080 256spp depth 8"
    for kind in ("bounce", "march"):
        k = rec["kinds"][kind]
        assert 1 <= k["mean_active_lanes"] <= 64 and k["algorithmic_flops_per_sample"] > 0
