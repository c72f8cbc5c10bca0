"""The PMC traffic tools (round 6): per-step bytes from FETCH_SIZE / WRITE_SIZE passes skip the
first stitch of the run and divide by the stitches that remain.  Round 5's table divided three
stitches by two because the one-launch projection (cyl_tile) was missing from the class
patterns, so every class read 1.5x its bytes (profiles/r06_pmc_correction_note.txt).  CPU only:
synthetic counter CSVs in rocprofv3's layout."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size",
          "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
          "Accum_VGPR_Count", "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]

# one parrington-shaped stitch: projection, gray, base, one level, extrema, localize
STITCH = [
    ("void (anonymous namespace)::cyl_tile<true>(unsigned char const*)", 100.0, 50.0),
    ("(anonymous namespace)::gray_frames(unsigned char const*)", 5200.0, 3466.0),
    ("void (anonymous namespace)::blur_fast<0, 11, 112, 64, 512>((anonymous namespace)::LoadArgs)", 1728.0, 55296.0),
    ("void (anonymous namespace)::blur_fast<1, 11, 112, 64, 512>((anonymous namespace)::LoadArgs)", 27648.0, 110592.0),
    ("void (anonymous namespace)::extrema_stream<5, 32>((anonymous namespace)::XArgs)", 1000.0, 10.0),
    ("(anonymous namespace)::localize((anonymous namespace)::DogArgs)", 300.0, 1.0),
]


def _write(root, counter, stitches, idx):
    d = os.path.join(root, counter)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, FIELDS)
        w.writeheader()
        i = 0
        for _ in range(stitches):
            for name, fetch, write in STITCH:
                i += 1
                row = {k: "0" for k in FIELDS}
                row.update(Dispatch_Id=str(i), Kernel_Name=name, Counter_Name=counter,
                           Counter_Value=str(fetch if idx == 0 else write), Start_Timestamp="0",
                           End_Timestamp="1000")
                w.writerow(row)


def test_pmc_traffic_skips_the_first_stitch(tmp_path):
    for k, c in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
        _write(str(tmp_path), c, 3, k)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path), "3",
                          "parrington"], capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    assert d["steps"] == 2
    blur = d["classes"]["blur_level"]
    assert blur["launches_per_step"] == 3.0                      # gray + base + one level
    want_r = 2 * (5200.0 + 1728.0 + 27648.0) * 1024
    want_w = (3466.0 + 55296.0 + 110592.0) * 1024
    assert blur["read_bytes_per_step"] == round(want_r) and blur["write_bytes_per_step"] == round(want_w)
    assert d["classes"]["cyl_scatter"]["launches_per_step"] == 1.0


def test_pmc_traffic_refuses_a_miscounted_trace(tmp_path):
    for k, c in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
        _write(str(tmp_path), c, 3, k)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path), "4",
                        "parrington"], capture_output=True, text=True)
    assert r.returncode != 0 and "stitches found" in r.stderr


def test_pmc_per_launch_names_the_planes(tmp_path):
    for k, c in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
        _write(str(tmp_path), c, 3, k)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_per_launch.py"), str(tmp_path), "3",
                          "parrington"], capture_output=True, text=True, check=True).stdout
    assert "o0 base: gray -> G0" in out and "o0 L1: G0 -> G1 + DoG0" in out
    assert "2 stitches averaged" in out
