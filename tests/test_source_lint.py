"""Source checks on the host -> device argument structs (no GPU).

The launch structs of src/device/kernels.h (KArgs, GradArgs, ...) are filled field by field on
the host and passed by value to the kernels.  A field a call site forgets must read as 0 / null,
never as stack garbage: round 5's GPU failure was GradArgs::write_split left uninitialised at
one call site (the kernel then skipped its grad / hess stores on a fresh box).  So every field
carries a default member initialiser, and no call site declares one of these structs without
value-initialising it.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARG_STRUCTS = {
    "src/device/kernels.h": ["KArgs", "DevTree", "PeerBufs", "PeerArgs", "GradArgs", "RankArgs", "SampleArgs",
                             "ForestArgs", "MetricArgs", "RenewArgs"],
    "src/device/device_types.h": ["Params"],
}


def _struct_fields(text, name):
    m = re.search(r"^struct (?:alignas\(\d+\) )?" + name + r" \{\n(.*?)^\};", text, re.S | re.M)
    assert m, name
    fields = []
    for ln in m.group(1).split("\n"):
        s = ln.strip()
        if not s or s.startswith("//") or ";" not in s:
            continue
        decl = s.split(";")[0]
        if "(" in decl:  # (member functions)
            continue
        fields.append(decl)
    return fields


def test_every_argument_struct_field_has_a_default_initialiser():
    missing = []
    for path, names in ARG_STRUCTS.items():
        text = open(os.path.join(ROOT, path)).read()
        for name in names:
            fields = _struct_fields(text, name)
            assert fields, name
            for decl in fields:
                for part in decl.split(","):
                    if "{}" not in part and "=" not in part:
                        missing.append("%s::%s" % (name, part.strip()))
    assert not missing, "fields without a default member initialiser: %s" % missing


def test_no_call_site_declares_an_argument_struct_uninitialised():
    names = [n for ns in ARG_STRUCTS.values() for n in ns]
    pat = re.compile(r"\b(?:dev::)?(" + "|".join(names) + r")\s+\w+\s*;")
    bad = []
    for d, _, files in os.walk(os.path.join(ROOT, "src")):
        for f in files:
            if not f.endswith((".cpp", ".hip", ".h")):
                continue
            p = os.path.join(d, f)
            for i, ln in enumerate(open(p, errors="replace"), 1):
                code = ln.split("//")[0]
                if pat.search(code) and "struct " not in code:
                    bad.append("%s:%d: %s" % (os.path.relpath(p, ROOT), i, ln.strip()))
    assert not bad, "argument structs declared without {}: %s" % bad
