"""The environment knobs: include/lgbm_amd/tuning.h is the only place the native library reads
LGBM_AMD_* variables from, and docs/ENVIRONMENT.md documents the same set."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table():
    hdr = open(os.path.join(ROOT, "include", "lgbm_amd", "tuning.h")).read()
    return set(re.findall(r'X\(\w+, "(LGBM_AMD_\w+)"', hdr))


def test_sources_read_knobs_only_through_tuning_header():
    offenders = []
    for d, _, files in list(os.walk(os.path.join(ROOT, "src"))) + list(os.walk(os.path.join(ROOT, "include"))):
        for f in files:
            if f.endswith((".cpp", ".hip", ".h")):
                text = open(os.path.join(d, f)).read()
                for m in re.finditer(r'getenv\("(LGBM_AMD_\w+)"\)', text):
                    offenders.append((f, m.group(1)))
    assert offenders == []


def test_environment_doc_matches_tuning_table():
    table = _table()
    doc = set(re.findall(r"`(LGBM_AMD_[A-Z0-9_]+)[`=]", open(os.path.join(ROOT, "docs", "ENVIRONMENT.md")).read()))
    # (DEVICE_COMM is read by the Python package)
    python_side = {"LGBM_AMD_DEVICE_COMM", "LGBM_AMD_KNOBS"}  # (KNOBS: the table macro itself)
    assert table - doc == set(), "undocumented: %s" % sorted(table - doc)
    assert doc - table - python_side == set(), "documented but not in tuning.h: %s" % sorted(doc - table - python_side)
