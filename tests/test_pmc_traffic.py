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


def _profile(root, rnd, name, workload, source, **extra):
    d = root / "profiles" / rnd
    d.mkdir(parents=True, exist_ok=True)
    rec = {"workload": workload, "source_id": source, "kinds": {"bounce": {"launches": 10, "traffic": 100.0,
                                                                           "algorithmic_flops_per_sample": 1.0}}}
    rec.update(extra)
    (d / name).write_text(json.dumps(rec))


def test_pmc_lookup_keys_on_scene_depth_and_build(tmp_path):
    """bench.py takes a committed PMC pass of the same (scene, depth, build) for any frame size and spp (FLOPs and
    bytes per sample are per-sample quantities): the exact workload first, then the newest round; other builds,
    scenes or depths never."""
    import bench
    _profile(tmp_path, "r3", "pmc_flops_c2.json", "cornell_box.json 1920x1080 256spp depth 8", "b1")
    _profile(tmp_path, "r3", "pmc_flops_c3.json", "cornell_box.json 3840x2160 1024spp depth 8", "b1")
    _profile(tmp_path, "r4", "pmc_flops_c2.json", "cornell_box.json 1920x1080 256spp depth 8", "b2")
    _profile(tmp_path, "r4", "pmc_flops_d50.json", "cornell_box.json 1920x1080 256spp depth 50", "b1")
    _profile(tmp_path, "r3", "pmc_flops_c5.json", "synthetic_100000 1920x1080 256spp depth 8", "b1")
    look = lambda *a: bench.pmc_lookup("flops", *a, root=tmp_path)  # noqa: E731
    f, rec, spf, why = look("cornell_box.json", 8, 3840, 2160, 1024, "b1")
    assert f.name == "pmc_flops_c3.json" and spf == 3840 * 2160 * 1024 and why is None  # exact workload
    f, rec, spf, why = look("cornell_box.json", 8, 3840, 2160, 4096, "b1")  # C4: no pass of its own
    assert rec["source_id"] == "b1" and rec["workload"].endswith("depth 8")
    f, rec, spf, why = look("cornell_box.json", 8, 3840, 2160, 4096, "b2")
    assert f.parent.name == "r4" and f.name == "pmc_flops_c2.json"
    f, rec, spf, why = look("cornell_box.json", 8, 1920, 1080, 256, "b9")
    assert rec is None and "b9" in why and "b1" in why
    f, rec, spf, why = look("cornell_box.json", 50, 1920, 1080, 256, "b1")
    assert f.name == "pmc_flops_d50.json"
    f, rec, spf, why = look("spheres.json", 8, 256, 256, 16, "b1")
    assert rec is None and "no committed" in why


def test_traffic_per_sample_is_frame_size_independent(tmp_path):
    """The pass's bytes per sample (launches x bytes per launch / its samples) are what a C4 or a rank's share is
    priced with: the frames key of a multi-frame pass divides them."""
    import bench
    wl = "cornell_box.json 1920x1080 256spp depth 8"
    _profile(tmp_path, "r4", "pmc_traffic_c2.json", wl, "b1", frames=2)
    f, rec, spf, why = bench.pmc_lookup("traffic", "cornell_box.json", 8, 3840, 2160, 4096, "b1", root=tmp_path)
    k = rec["kinds"]["bounce"]
    per_sample = k["traffic"] * k["launches"] / (spf * rec.get("frames", 1))
    assert per_sample == 100.0 * 10 / (1920 * 1080 * 256 * 2)


def test_committed_passes_serve_every_cornell_config():
    """Every committed C2/C3 pass is a cornell depth-8 workload bench.py can key on; C4 (no pass of its own) finds
    one of them for whatever build they were collected on."""
    import bench
    for rnd in ("r3", "r4"):
        for f in sorted((ROOT / "profiles" / rnd).glob("pmc_*_c[23].json")):
            rec = json.loads(f.read_text())
            wl = bench.parse_workload(rec["workload"])
            assert wl and wl[0] == "cornell_box.json" and wl[4] == 8, f
            f2, rec2, _, why = bench.pmc_lookup(f.name.split("_")[1], "cornell_box.json", 8, 3840, 2160, 4096,
                                                rec["source_id"])
            assert rec2 is not None and rec2["source_id"] == rec["source_id"], why


def test_f32_node_flops_per_sample():
    """The large-tree bounce's f32 node work for the roofline's valu_f32 part: 12 FLOPs per node test, less the
    root test its walk skips once per trace (C5 host count: 120.6 node tests and 2.73 traces per sample)."""
    import bench
    counts = {"samples": 1000, "node_slabs": 120596, "bounces": 2731}
    assert abs(bench.f32_node_flops_per_sample(counts) - 12 * (120596 - 2731) / 1000) < 1e-9
    assert bench.f32_node_flops_per_sample({"samples": 0, "node_slabs": 0, "bounces": 0}) == 0.0
