"""Profiling tools on synthetic inputs: the kernel-class grouping of a
prof_summary table and the per-step HBM byte table from rocprofv3 --pmc CSVs (the marker
window, FETCH_SIZE x 2 calibration, per-class and per-kernel rows)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")
sys.path.insert(0, TOOLS)


def test_kernel_classes_assignment():
    from kernel_classes import CLASSES
    import re

    def cls(name):
        for c, pat in CLASSES:
            if re.search(pat, name):
                return c
        return None

    assert cls("void cml::(anonymous namespace)::conv3x3p_kernel<1>(P3Args)").startswith("3x3 conv fwd")
    assert cls("void cml::(anonymous namespace)::gemm_nt_kernel<3, true>(cml::GemmArgs)").startswith(
        "3x3 conv fwd")
    assert cls("void cml::(anonymous namespace)::gemm_nt_kernel<0, false>(cml::GemmArgs)").startswith(
        "own GEMM")
    assert cls("void cml::(anonymous namespace)::wgrad3x3_kernel<64>(W3Args)").startswith("3x3 weight")
    assert cls("igemm_wrw_gtcx35_nhwc_bf16_bx0_ex0_bt256x256x32").startswith("conv wgrad")
    assert cls("Cijk_Ailk_Bjlk_BBS_BH_Bias_HA_S_SAV_UserArgs_MT256x256x32") == "GEMM (hipBLASLt)"


def test_kernel_classes_table(tmp_path):
    md = tmp_path / "k.md"
    md.write_text("| kernel | calls | total ms | avg us | % | ms/step |\n|---|---|---|---|---|---|\n"
                  "| `void cml::(anonymous namespace)::conv3x3p_kernel<1>(x)` | 6 | 3.0 | 500 | 50 | 1.5 |\n"
                  "| `igemm_wrw_gtcx35_nhwc_bf16` | 6 | 2.0 | 300 | 30 | 1.0 |\n"
                  "| `__amd_rocclr_fillBufferAligned` | 6 | 0.2 | 30 | 20 | 0.1 |\n")
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "kernel_classes.py"), str(md)],
                         capture_output=True, text=True, check=True).stdout
    assert "| 1.50 |" in out and "| 1.00 |" in out and "total (listed kernels) | 2.60" in out


def _write_csv(path, counter, rows):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value",
                    "Start_Timestamp", "End_Timestamp"])
        for i, (name, val, ns) in enumerate(rows):
            w.writerow([i + 1, 1024, name, counter, val, 1000 * i, 1000 * i + ns])


def test_pmc_step_bytes(tmp_path):
    k = "void cml::(anonymous namespace)::conv3x3p_kernel<1>(x)"
    # before the marker (ignored), the marker, then two steps of one kernel
    rows_f = [(k, 1e9, 10), ("spin_kernel", 0.0, 10), (k, 1e6, 500_000), (k, 1e6, 500_000)]
    rows_w = [(k, 1e9, 10), ("spin_kernel", 0.0, 10), (k, 5e5, 500_000), (k, 5e5, 500_000)]
    _write_csv(tmp_path / "f", "FETCH_SIZE", rows_f)
    _write_csv(tmp_path / "w", "WRITE_SIZE", rows_w)
    tool = os.path.join(TOOLS, "pmc_step_bytes.py")
    out = subprocess.run([sys.executable, tool, "--steps", "2", str(tmp_path / "f"),
                          str(tmp_path / "w")], capture_output=True, text=True, check=True).stdout
    # per step: read 2 x 1e6 KiB (FETCH x 2), written 5e5 KiB
    gb_r, gb_w = 2 * 1e6 * 1024 / 1e9, 5e5 * 1024 / 1e9
    assert f"| {gb_r:.1f} | {gb_w:.1f} | {gb_r + gb_w:.1f} |" in out
    out = subprocess.run([sys.executable, tool, "--steps", "2", "--per-kernel", "5",
                          str(tmp_path / "f"), str(tmp_path / "w")],
                         capture_output=True, text=True, check=True).stdout
    # one group: GB / step, 0.5 ms / step, TB/s = GB / ms
    line = [ln for ln in out.splitlines() if "conv3x3p" in ln][0]
    cells = [c.strip() for c in line.strip("|").split("|")]
    assert cells[2] == "1" and abs(float(cells[4]) - 0.5) < 1e-3
    assert abs(float(cells[5]) - float(cells[3]) / 0.5) < 0.02
