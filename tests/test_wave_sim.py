"""tools/wave_sim.py — the lock-step wave simulation of the lane tree walk that
sized round 6's step changes — still builds against the
product's tree_walk.h (it patches a copy at fixed anchors) and gives the
counts its design notes quote: config 4 at 9.2 wave steps per 64 traces with
its one close site and one draw site, every wave step of c3p running all three
draw sites.  CPU only (g++)."""
import os
import re
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT


def run(config, *defs, traces=2000):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    args = [sys.executable, os.path.join(ROOT, "tools", "wave_sim.py"), "--config", config, "--traces", str(traces)]
    for d in defs:
        args += ["-D", d]
    out = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr + out.stdout
    steps = float(re.search(r"wave_steps_per_64 ([0-9.]+)", out.stdout).group(1))
    sites = {m.group(1): (float(m.group(2)), float(m.group(3)))
             for m in re.finditer(r"^\s+(\S+)\s+wave steps ([0-9.]+)\s+lane-steps ([0-9.]+)", out.stdout, re.M)}
    return steps, sites


def test_config4_steps_and_sites():
    steps, sites = run("c4")
    assert 8.0 < steps < 10.5, steps
    assert sites["res_open"][0] > 0.9 and sites["err_blk"][0] == 0.0  # no error draws on config 4
    assert sites["close"][0] > 0.9


def test_c3p_every_draw_site_every_step():
    steps, sites = run("c3p", traces=640)
    for s in ("res_kb", "err_blk", "res_open"):
        assert sites[s][0] > 0.95 and sites[s][1] < 0.5, (s, sites[s])  # the wave runs it; few lanes need it
    # a smaller scan budget makes more steps (the same walk: results equal, tests/test_tree_walk.py)
    steps2, _ = run("c3p", "TW_SCAN=1", traces=640)
    assert steps2 > steps
