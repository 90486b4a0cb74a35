"""Guard the compiled step kernels' resource budget and LDS-wait schedule on the CPU box.

The step kernel runs at 2 waves per SIMD (an env pair per wave, every 4096-env wave resident) with its
VGPRs a few registers from the 256 cliff, and part of its speed rests on `asm volatile` pins that
batch LDS reads behind one wait (DESIGN.md §3 "LDS waits").  A compiler or source change that spills,
drops occupancy, grows LDS past 8 workgroups per CU or re-exposes the LDS latencies would silently
cost throughput; this test compiles allsteps_kernels.hip with the package's own flags
(_native.STEP_FLAGS) and holds it to tests/kernel_budget.json."""

import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")


@pytest.fixture(scope="module")
def compiled(tmp_path_factory):
    from allsteps_isaaclab_amd import _native

    d = tmp_path_factory.mktemp("kbudget")
    asm = d / "k.s"
    r = subprocess.run([HIPCC, *_native.STEP_FLAGS, "--cuda-device-only", "-S", "-o", str(asm),
                        "-Rpass-analysis=kernel-resource-usage", os.path.join(_native.CSRC, "allsteps_kernels.hip")],
                       capture_output=True, text=True, timeout=600, cwd=str(d))
    assert r.returncode == 0, r.stderr[-3000:]
    res, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line)
        if m:
            cur = res.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+([A-Za-z][A-Za-z /\[\]]*?):\s+(\S+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    return res, asm.read_text().split("\n")


BUDGET = {k: v for k, v in json.load(open(os.path.join(ROOT, "tests", "kernel_budget.json"))).items()
          if k != "_comment"}


@pytest.mark.parametrize("func", sorted(BUDGET))
def test_step_kernel_resources(compiled, func):
    res, _ = compiled
    b, r = BUDGET[func], res[func]
    print(func, r)
    assert int(r["VGPRs"]) <= b["vgpr_max"], r
    assert int(r["AGPRs"]) <= b["agpr_max"], r
    assert int(r["ScratchSize [bytes/lane]"]) <= b["scratch_max"], r
    assert int(r["VGPRs Spill"]) == 0, r
    assert int(r["SGPRs Spill"]) <= b["sgpr_spill_max"], r
    assert int(r["LDS Size [bytes/block]"]) <= b["lds_max"], r
    assert int(r["Occupancy [waves/SIMD]"]) == b["occupancy"], r


@pytest.mark.parametrize("func", sorted(BUDGET))
def test_step_kernel_lds_waits(compiled, func):
    import lgkm_stalls

    _, lines = compiled
    hits = lgkm_stalls.scan(lines, func, 8)
    print(f"{func}: {len(hits)} early LDS waits")
    assert len(hits) <= BUDGET[func]["early_lds_waits_max"], hits[:20]
