"""The drop-in library reads its NGT_AMD_* tuning variables only through
knob() (ngt_amd/csrc/knobs.h), which answers only with NGT_AMD_TEST_KNOBS=1:
no other environment read in the product sources may name an NGT_AMD_
variable, except the public NGT_AMD_DEVICE."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ngt_amd", "csrc")


def test_no_raw_knob_reads():
    bad = []
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith((".cpp", ".hip", ".h")) or f == "knobs.h":
            continue
        for i, line in enumerate(open(os.path.join(CSRC, f)), 1):
            for m in re.finditer(r'getenv\("(NGT_AMD_[A-Z0-9_]*)"\)', line):
                if m.group(1) != "NGT_AMD_DEVICE":
                    bad.append("%s:%d %s" % (f, i, m.group(1)))
    assert not bad, bad


def test_knob_table_documented():
    """Every knob the library reads is in DESIGN.md's knob table."""
    names = set()
    for f in os.listdir(CSRC):
        if f.endswith((".cpp", ".hip", ".h")):
            names |= set(re.findall(r'knob\("(NGT_AMD_[A-Z0-9_]*)"\)', open(os.path.join(CSRC, f)).read()))
    design = open(os.path.join(ROOT, "DESIGN.md")).read()
    missing = sorted(n for n in names if n not in design)
    assert names and not missing, missing
