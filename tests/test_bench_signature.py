"""bench.py keys the PMC profile it reports (profiles/pmc_latest.json) to a signature of the
likelihood kernel's code: comment edits keep it, code edits change it."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _reader(edit):
    def read(rel):
        with open(os.path.join(ROOT, rel), encoding="utf-8") as f:
            text = f.read()
        return edit(rel, text)
    return read


def test_signature_ignores_comments_not_code():
    base = bench.kernel_signature()
    assert base == bench.kernel_signature(read=_reader(lambda rel, t: t))
    commented = _reader(lambda rel, t: t.replace("namespace rvm {", "// a note\nnamespace rvm { /* another */", 1)
                        if rel.endswith("rvm_logl.hip") else t)
    assert bench.kernel_signature(read=commented) == base
    changed = _reader(lambda rel, t: t.replace("RVM_LS_RING = 64", "RVM_LS_RING = 63", 1)
                      if rel.endswith("rvm_internal.h") else t)
    assert bench.kernel_signature(read=changed) != base
