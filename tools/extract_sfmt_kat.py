#!/usr/bin/env python3
"""Extract the SFMT-19937 known-answer vector of the reference's own test
(src/tests/test_random.cpp:433-507: 192 nextULong() outputs of Random(4321))
into tests/golden/sfmt_seed4321.json.  Reads the reference as DATA only;
the committed fixture is what the tests use."""
import json, os, re
src = open("/root/reference/src/tests/test_random.cpp").read()
block = src[src.index("static const uint64_t reference[]"):]
block = block[:block.index("};")]
vals = [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]+)ULL", block)]
assert len(vals) == 192, len(vals)
out = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "sfmt_seed4321.json")
json.dump({"source": "reference src/tests/test_random.cpp:433-507 (TestRandom::test00_validate)",
           "seed": 4321, "next_ulong": [str(v) for v in vals]}, open(out, "w"), indent=1)
print("wrote", len(vals))
