"""Regenerates the committed fixtures that come from running the reference's
own Python generator (run in the build container, where /root/reference is
mounted; the GPU box only reads the committed outputs).

* topologies/gen-tree-4x8-concurrent.yaml: isotope/create_tree_topology.py
  with NUM_LEVELS=4, NUM_BRANCHES=8 (module constants patched after import,
  NUM_SERVICES recomputed as the script's line 32 does), main() run in a
  temporary directory; its gen.yaml is copied verbatim.
"""
import importlib.util
import os
import shutil
import sys
import tempfile

REF = "/root/reference/isotope/create_tree_topology.py"
HERE = os.path.dirname(os.path.abspath(__file__))


def tree_fixture(levels=4, branches=8):
    spec = importlib.util.spec_from_file_location("create_tree_topology", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.NUM_LEVELS = levels
    mod.NUM_BRANCHES = branches
    mod.NUM_SERVICES = sum(branches ** i for i in range(levels))
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            mod.main()
        finally:
            os.chdir(cwd)
        out = os.path.join(HERE, "topologies", f"gen-tree-{levels}x{branches}-concurrent.yaml")
        shutil.copy(os.path.join(d, "gen.yaml"), out)
    return out


if __name__ == "__main__":
    print(tree_fixture(4, 8))
    print(tree_fixture(3, 3))
    sys.exit(0)
