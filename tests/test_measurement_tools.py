"""The measurement tools on synthetic inputs (CPU): tools/pmc_traffic.py's
per-pass normalisation (two rocprofv3 passes whose runs differ by a launch)
and tools/sq_summary.py's shares."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size", "Kernel_Id",
          "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count",
          "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]


def write_counters(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(HEADER)
        for d, kernel, name, value in rows:
            w.writerow([d, d, "Agent 2", 1, 1, 1, 64, 1, kernel, 64, 0, 0, 64, 0, 32, name, value, 0, 1])


def bench_line(path, run):
    with open(path, "w") as f:
        f.write(json.dumps({"run_estep_log": run}) + "\n")


def test_pmc_traffic_each_pass_over_its_own_run(tmp_path):
    k = "void hmc::estep_values<false, 4, false, true>(hmc::ValueArgs)"
    # fetch run: 3 launches over R_E = 100 + 50 (8 B each); write run: 2 launches over R_E = 150
    write_counters(tmp_path / "f.csv", [(1, k, "FETCH_SIZE", 1.0), (2, k, "FETCH_SIZE", 2.0), (3, k, "FETCH_SIZE", 3.0),
                                        (4, "other", "FETCH_SIZE", 1e9)])
    write_counters(tmp_path / "w.csv", [(1, k, "WRITE_SIZE", 4.0), (2, k, "WRITE_SIZE", 5.0)])
    bench_line(tmp_path / "bf.json", [[100, 2], [50, 1]])
    bench_line(tmp_path / "bw.json", [[150, 2]])
    out = tmp_path / "o.json"
    subprocess.check_call([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path / "f.csv"),
                           str(tmp_path / "w.csv"), "estep_values", str(out), "cmd", str(tmp_path / "bf.json"),
                           str(tmp_path / "bw.json")], stdout=subprocess.DEVNULL)
    d = json.load(open(out))
    alg = 8.0 * 150
    assert d["launches"] == 3 and d["alg_launches"] == 3 and d["alg_launches_write_run"] == 2
    assert d["launches_match"]
    assert abs(d["fetch_x2_over_alg"] - 2 * 6 * 1024 / alg) < 1e-12
    assert abs(d["write_over_alg"] - 9 * 1024 / alg) < 1e-12
    assert abs(d["traffic_over_alg"] - (12 + 9) * 1024 / alg) < 1e-12
    assert abs(d["traffic_over_alg_raw_fetch"] - (6 + 9) * 1024 / alg) < 1e-12


def test_sq_summary_shares(tmp_path):
    k = "void hmc::estep_values<false, 5, false, true>(hmc::ValueArgs)"
    write_counters(tmp_path / "a.csv", [(1, k, "SQ_WAVE_CYCLES", 100.0), (1, k, "SQ_WAIT_ANY", 40.0),
                                        (1, k, "SQ_WAIT_INST_ANY", 25.0), (1, k, "SQ_ACTIVE_INST_ANY", 35.0),
                                        (1, k, "SQ_INSTS_VALU", 2e12), (1, k, "SQ_INSTS_SALU", 5e11)])
    write_counters(tmp_path / "b.csv", [(1, k, "SQ_INSTS_LDS", 3e11), (1, k, "SQ_LDS_BANK_CONFLICT", 50.0),
                                        (1, k, "SQ_ACTIVE_INST_LDS", 100.0)])
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), str(tmp_path / "a.csv"),
                        str(tmp_path / "b.csv")], capture_output=True, text=True, check=True)
    row = [ln for ln in r.stdout.splitlines() if "estep_values<false, 5" in ln][0]
    assert "| 40 % | 25 % | 35 % | 2.00 : 0.50" in row and "| 50 % |" in row


def test_sq_summary_issue_fraction_json(tmp_path):
    """valu_issue_frac = SQ_INSTS_VALU * 4 / (1024 SIMDs * 2.4 GHz * kernel seconds of the pass);
    the JSON carries the profiled run's library identity for bench.py's same-build check."""
    k = "void hmc::estep_values<false, 4, false, true>(hmc::ValueArgs)"
    write_counters(tmp_path / "a.csv", [(1, k, "SQ_WAVE_CYCLES", 100.0), (1, k, "SQ_INSTS_VALU", 2.4e3),
                                        (2, k, "SQ_INSTS_VALU", 2.4e3)])
    write_counters(tmp_path / "b.csv", [(1, k, "SQ_LDS_BANK_CONFLICT", 30.0), (1, k, "SQ_ACTIVE_INST_LDS", 60.0)])
    with open(tmp_path / "bench.json", "w") as f:
        f.write("progress\n" + json.dumps({"library": {"sha256_16": "abc"}}) + "\n")
    out = tmp_path / "sq.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), str(tmp_path / "a.csv"),
                    str(tmp_path / "b.csv"), "estep_values", str(out), str(tmp_path / "bench.json")],
                   capture_output=True, text=True, check=True)
    d = json.load(open(out))
    kk = d["kernels"]["hmc::estep_values<false, 4, false, true>"]
    assert kk["launches"] == 2 and abs(kk["kernel_seconds"] - 2e-9) < 1e-18
    assert abs(kk["valu_issue_frac_nominal"] - 4 * 4.8e3 / (1024 * 2.4e9 * 2e-9)) < 1e-9
    assert kk["valu_issue_frac"] is None  # no busy pass: nothing measured
    assert abs(kk["lds_bank_conflict_ratio"] - 0.5) < 1e-12
    assert d["library"] == {"sha256_16": "abc"}


def test_sq_summary_measured_issue_with_dual_issue(tmp_path):
    """Measured VALU issue (round 6): one instruction per quad-cycle per SIMD,
    two when they dual-issue (SQ_ACTIVE_INST_VALU2 quad-cycles), over 32 SIMDs
    per shader engine x SQ_BUSY_CYCLES (summed over the engines):
    4 * (VALU - VALU2) / (32 * BUSY); the mix pass gives per-type shares."""
    k = "void hmc::estep_values<false, 4, false, true>(hmc::ValueArgs)"
    write_counters(tmp_path / "a.csv", [(1, k, "SQ_WAVE_CYCLES", 100.0), (1, k, "SQ_INSTS_VALU", 1e6)])
    write_counters(tmp_path / "b.csv", [(1, k, "SQ_LDS_BANK_CONFLICT", 1.0), (1, k, "SQ_ACTIVE_INST_LDS", 2.0)])
    write_counters(tmp_path / "busy.csv", [(1, k, "SQ_INSTS_VALU", 1000.0), (1, k, "SQ_ACTIVE_INST_VALU2", 100.0),
                                           (1, k, "SQ_BUSY_CYCLES", 50.0)])
    write_counters(tmp_path / "mix.csv", [(1, k, "SQ_INSTS_VALU", 1000.0), (1, k, "SQ_INSTS_VALU_INT32", 450.0),
                                          (1, k, "SQ_INSTS_VALU_ADD_F64", 10.0)])
    with open(tmp_path / "bench.json", "w") as f:
        f.write(json.dumps({"library": {"sha256_16": "abc"}}) + "\n")
    out = tmp_path / "sq.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), str(tmp_path / "a.csv"),
                    str(tmp_path / "b.csv"), "estep_values", str(out), str(tmp_path / "bench.json"),
                    str(tmp_path / "busy.csv"), str(tmp_path / "mix.csv")], capture_output=True, text=True, check=True)
    kk = json.load(open(out))["kernels"]["hmc::estep_values<false, 4, false, true>"]
    assert kk["valu_issue_frac"] == 4 * (1000 - 100) / (32 * 50.0)
    assert kk["valu_dual_issue_share"] == 0.2 and kk["valu_cycles_per_inst"] == 3.6
    assert kk["valu_mix"]["INT32"] == 0.45 and kk["valu_mix"]["ADD_F64"] == 0.01
    sys.path.insert(0, ROOT)
    import bench
    d = json.load(open(out))
    d["library"] = {"sha256_16": "abc"}
    os.makedirs(tmp_path / "p", exist_ok=True)
    with open(tmp_path / "p" / "sq_estep_values_cfgX.json", "w") as f:
        json.dump(d, f)
    old = bench.PMC_DIRS
    try:
        bench.PMC_DIRS = [str(tmp_path / "p")]
        sq = bench.sq_summary("cfgX", {"sha256_16": "abc"})
    finally:
        bench.PMC_DIRS = old
    assert sq["same_build"] and sq["valu_issue_frac"] == kk["valu_issue_frac"] and sq["valu_dual_issue_share"] == 0.2
