"""bench.py's BASELINE config-3 lines on a small batch, on the GPU: the Get
as Client.decode runs it (client/ecRedis.go:404-427), fused (dec4_get) and
unfused (dec4_upstream).  Each line names the kernel the library runs
(gf_apply_tri for these shapes), proves its work (garbage into the rebuilt
rows, bit-exact compare) and its checks (one corrupted byte of an extra
parity shard flags exactly its object), and carries a CPU leg that runs the
Go path's Reconstruct + Verify, bit-exact against the GPU."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(workload):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", workload, "--batch", "16",
           "--steps", "2", "--warmup", "1", "--cpu-seconds", "1", "--no-pmc"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("workload,kernel", [("dec4_get", "gf_apply_tri<12,4>"),
                                             ("dec4_upstream", "gf_apply_tri<14,4>")])
def test_config3_get_lines(gpu, workload, kernel):
    out = _line(workload)
    assert out["config"]["k"] == 10 and out["config"]["p"] == 4 and out["config"]["batch_per_gpu"] == 16
    r = out["roofline"]
    assert r["kernel"].startswith(kernel) and 0 < r["frac"] < 1
    wc = out["work_check"]["decode"]
    assert wc["result"] == "bit-exact" and wc["rows_rewritten"] == 32
    assert wc["corruption_check"]["flagged"] == [8] and wc["corruption_check"]["row"] == 13
    cpu = out["cpu_baseline"]
    assert "Reconstruct then Verify" in cpu["decode_form"] and cpu["sample"].endswith(": True")
    if workload == "dec4_get":
        assert cpu["fused_form_GiBps"] > 0
        # 12 rows read + 2 written per object
        assert r["kernel"].split("), ")[1].startswith(str(16 * 14 * ((4 << 20) // 10 + 1)))
    else:
        assert set(r["kernel_ms_alone"]) == {"decode:reconstruct", "decode:verify"}
