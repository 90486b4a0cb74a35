"""Dev tooling: scripts/lgkm_stalls.py (the static scan that located the exposed LDS waits, DESIGN §3
"LDS waits") on a synthetic kernel listing."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ASM = """\
_Z4kernv:
\tds_read_b128 v[0:3], v10
\tds_read_b128 v[4:7], v10 offset:16
\ts_waitcnt lgkmcnt(1)
\tv_add_f32_e32 v8, v0, v1
.LBB0_1:
\tds_read_b32 v9, v11
\tv_mov_b32_e32 v12, v13
\tv_mov_b32_e32 v14, v15
\tv_mov_b32_e32 v16, v17
\tv_mov_b32_e32 v18, v19
\tv_mov_b32_e32 v20, v21
\tv_mov_b32_e32 v22, v23
\tv_mov_b32_e32 v24, v25
\tv_mov_b32_e32 v26, v27
\ts_waitcnt lgkmcnt(0)
\tv_add_f32_e32 v8, v9, v4
.Lfunc_end0:
"""


def test_lgkm_stalls_reports_only_early_waits(tmp_path):
    f = tmp_path / "k.s"
    f.write_text(ASM)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "lgkm_stalls.py"), str(f), "--func", "_Z4kernv",
                        "--min", "6"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = [x for x in r.stdout.splitlines() if "waited" in x]
    # the first read is retired by lgkmcnt(1) two instructions after issue: reported; the second
    # read's block ends (a new block starts with nothing tracked), and the read in .LBB0_1 is waited
    # on nine instructions later: not reported
    assert len(lines) == 1, r.stdout
    assert "ds_read_b128 v[0:3], v10" in lines[0] and "waited 2 instructions" in lines[0]
    assert "1 early waits" in r.stderr
