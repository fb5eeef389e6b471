"""CPU check of the mode-B draw-stream close list (kernel kind 6): the host
program compiler's StreamClose records, applied the way walk_stream_cl applies
them (32-record chunks of error bits, the last erring position before the
chunk), must reproduce the direct definition of mode B on the stream (an
invocation responds 500 iff an invocation of its subtree erred) for random
error patterns: per-site 500 counts, per-trace 500 count and entry status.
The checker (tests/cpp/close_list_check.cpp) links the product's own loader
and program compiler, built here with g++."""
import glob
import json
import os
import shutil
import subprocess

import pytest

from isim.generators import config2_topology, config3_topology, realistic_topology
from isim.yamljson import obj_to_json, yaml_to_json

from conftest import TOPOLOGIES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "istio-isotope_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("clc") / "close_list_check")
    srcs = [os.path.join(ROOT, "tests", "cpp", "close_list_check.cpp")] + \
        [os.path.join(CSRC, f) for f in ("json.cpp", "gounits.cpp", "graph.cpp", "program.cpp")]
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), "-I", CSRC, *srcs,
                    "-o", out], check=True)
    return out


def _chain(n, fan):
    svcs = []
    for i in range(n):
        calls = [[{"call": f"c{i + 1}"}] + [{"call": f"l{i}-{j}"} for j in range(fan)]] if i + 1 < n else []
        svcs.append({"name": f"c{i}", "script": [{"sleep": "1us"}] + calls})
        svcs += [{"name": f"l{i}-{j}"} for j in range(fan)]
    svcs[0]["isEntrypoint"] = True
    return json.dumps({"services": svcs})


def _run(checker, tmp_path, text, rounds=40, permille=(3, 50, 400)):
    path = tmp_path / "g.json"
    path.write_text(text)
    for pm in permille:
        r = subprocess.run([checker, str(path), str(rounds), str(pm)], capture_output=True, text=True)
        if r.returncode == 3:
            return False  # no draw stream (a dynamic walk)
        assert r.returncode == 0, r.stderr + r.stdout
    return True


def test_config3_and_config2(checker, tmp_path):
    assert _run(checker, tmp_path, obj_to_json(config3_topology()), rounds=20)
    assert _run(checker, tmp_path, obj_to_json(config2_topology()))


@pytest.mark.parametrize("depth", [1, 2, 31, 32, 33, 64])
@pytest.mark.parametrize("fan", [0, 1, 7, 40])
def test_chains(checker, tmp_path, depth, fan):
    assert _run(checker, tmp_path, _chain(depth, fan))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_realistic_trees(checker, tmp_path, seed):
    # concurrent fan-out: mode B keeps the walk static (no call after a fallible call)
    d = realistic_topology(1000 * seed, "multitier", seed=seed, concurrent=True, sleep_ms=(1, 5),
                           error_rate=(0, 0.05))
    assert _run(checker, tmp_path, obj_to_json(d))


def test_reference_topologies(checker, tmp_path):
    ran = 0
    for p in sorted(glob.glob(os.path.join(TOPOLOGIES, "*.yaml"))):
        ran += _run(checker, tmp_path, yaml_to_json(open(p, "rb").read()))
    assert ran > 0
