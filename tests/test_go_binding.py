"""The committed cgo binding (go/isim/isim.go): every C
function and type it names is declared in include/isim.h.  Go is absent from
this image and from the GPU box; when a toolchain is present, `go vet` runs
too (it needs sigs.k8s.io/yaml v1.2.0 in the module cache)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "isim", "isim.go")
HDR = open(os.path.join(ROOT, "include", "isim.h")).read()


def test_go_uses_only_declared_c_symbols():
    src = open(GO).read()
    used = set(re.findall(r"\bC\.(isim_[a-z0-9_]+|ISIM_[A-Z0-9_]+)", src))
    assert used, "no C symbols found"
    missing = [u for u in sorted(used) if not re.search(r"\b%s\b" % re.escape(u), HDR)]
    assert not missing, missing
    # every function the ABI exports for serving / graphs / manifests has a Go entry point
    for fn in ("isim_graph_unmarshal_json", "isim_handler_create", "isim_serve", "isim_serve_des",
               "isim_graph_marshal_json", "isim_graph_to_dot", "isim_graph_to_k8s_manifests",
               "isim_graph_marshal_yaml", "isim_multi_init_all", "isim_multi_init_rank", "isim_serve_multi",
               "isim_multi_abort"):
        assert "C." + fn + "(" in src, fn


@pytest.mark.skipif(shutil.which("go") is None, reason="no Go toolchain in this image")
def test_go_vet():
    r = subprocess.run(["go", "vet", "./..."], cwd=os.path.join(ROOT, "go"), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
