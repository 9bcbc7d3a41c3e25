"""INTEGRATION.md's Rust `extern "C"` block names every entry point include/ans_capi.h declares
(the binding a reference maintainer adds must cover the whole drop-in boundary)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_binds_every_capi_entry():
    with open(os.path.join(ROOT, "include", "ans_capi.h")) as f:
        header = f.read()
    names = re.findall(r"^(?:int|void|const char \*|uint64_t|double)\s*\*?\s*(ans_\w+)\s*\(", header, re.M)
    assert len(names) > 80
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    bound = set(re.findall(r"pub fn (ans_\w+)\(", doc))
    assert not [n for n in names if n not in bound], "declared in include/ans_capi.h but not bound in INTEGRATION.md"
