"""Profiling tools on synthetic rocprofv3 outputs (no GPU): the PMC summary
(tools/pmc_summary.py) and the kernel-trace step splitter (tools/prof_db.py)."""
import csv
import os
import sqlite3
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")


def _pmc_csv(path, counter, per_call, kernels):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        d = 0
        for name, n in kernels:
            for _ in range(n):
                d += 1
                w.writerow({"Dispatch_Id": d, "Kernel_Name": name, "Counter_Name": counter,
                            "Counter_Value": per_call})


def test_pmc_summary_calls_per_run_and_bytes(tmp_path):
    ks = [("void hipserve::paged_decode_kernel<128, 4>(unsigned short*)", 32),
          ("Cijk_Alik_Bljk_BBS_BH_MT256x256x64_MI16x16x1", 4)]
    a, b = tmp_path / "p1.csv", tmp_path / "p2.csv"
    _pmc_csv(a, "FETCH_SIZE", 1024.0, ks)  # KiB per call
    _pmc_csv(b, "WRITE_SIZE", 10.0, ks)
    out = tmp_path / "s.md"
    r = subprocess.run([sys.executable, "pmc_summary.py", str(out), "t", str(a), str(b)], cwd=TOOLS,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    rows = {ln.split("|")[1].strip(): [c.strip() for c in ln.split("|")[2:-1]]
            for ln in out.read_text().splitlines() if ln.startswith("| `")}
    pd = rows["`hipserve::paged_decode_kernel<128, 4>`"]
    assert pd[0] == "32"  # dispatches of ONE run, not summed over the two passes
    # 2x FETCH_SIZE (gfx950 half-count) in KiB -> MB per call
    assert abs(float(pd[-1]) - 2 * 1024 * 1024 / 1e6) < 0.01
    assert rows["`hipBLASLt GEMM MT256x256x64`"][0] == "4"


def test_prof_db_splits_steps_at_sampler(tmp_path):
    db = tmp_path / "run_results.db"
    c = sqlite3.connect(db)
    c.execute("create table kernels (name text, start integer, end integer)")
    t = 0
    for step in range(4):
        for name in ["hipserve::decode_gemm_kernel<4>", "hipserve::paged_decode_kernel<128, 4>",
                     "hipserve::mc_final_kernel<unsigned short>"]:
            c.execute("insert into kernels values (?, ?, ?)", (name, t, t + 1000))
            t += 1500  # 500 ns idle after every kernel
    c.commit()
    c.close()
    sys.path.insert(0, TOOLS)
    try:
        import prof_db
    finally:
        sys.path.remove(TOOLS)
    steps = prof_db.steps(prof_db.load(str(db)))
    assert len(steps) == 4 and all(len(s) == 3 for s in steps)
    assert steps[0][-1][0].startswith("hipserve::mc_final_kernel")
