"""The ctypes signatures in ops/hip.py must match the C ABI of csrc/kernels (checked on CPU
by parsing the sources, so a mismatch never costs a GPU run)."""
import glob
import os
import re

from conftest import ROOT

_CTYPE = {"int": "i", "unsigned": "u", "float": "f", "long long": "ll", "double": "d"}


def _c_signatures():
    sigs = {}
    for path in glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")):
        src = open(path).read()
        for m in re.finditer(r"DBA_EXPORT\s+(?:int|long long)\s+(\w+)\s*\(([^)]*)\)", src, re.S):
            params = [p.strip() for p in m.group(2).split(",") if p.strip()]
            kinds = []
            for p in params:
                p = re.sub(r"\s+\w+$", "", p)          # drop the parameter name
                if "*" in p:
                    kinds.append("p")
                else:
                    p = p.replace("const", "").strip()
                    kinds.append(_CTYPE[p])
            sigs[m.group(1)] = kinds
    return sigs


def test_ctypes_signatures_match_c_abi():
    import ctypes
    src = open(os.path.join(ROOT, "dba_mod_amd", "ops", "hip.py")).read()
    start = src.index("_SIGS = {")
    block = src[start:src.index("}\n", start) + 1]
    env = {"_P": "p", "_I": "i", "_LL": "ll", "_F": "f", "_U": "u", "_D": "d"}
    table = eval(block.split("=", 1)[1], {}, env)
    c = _c_signatures()
    assert set(table) <= set(c), set(table) - set(c)
    for name, kinds in table.items():
        assert kinds == c[name], (name, kinds, c[name])
