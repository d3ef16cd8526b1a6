"""Regenerate tests/golden/manifest.json from the oracle and check it against the
reference values recorded in SURVEY.md (Appendix A hashes, §8c error known-answers,
Appendix C trace hashes).  Run: python tests/golden/make_manifest.py"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as O  # noqa: E402

# SURVEY.md Appendix A (output SHA-256 of each fixture, reference src/inflate.c at -16)
SURVEY_OUT = {
    "100k_lines": ("821aaf56d797799dc619d506cb8a9e70a21257898843ce13e71a5474da7ced0b", 2188890),
    "10k_lines": ("261971e26d8aaf26d9ab10225d64ab23da555b5d85de847fd6ce5edafbaa910d", 120000),
    "payload_63k": ("6a95277fe915a852df57f872d9f9c0863777626dfd68d9e418242fc26973dbd0", 64512),
    "payload_64k": ("9b839dd63b8ce0258e03f87b1c8c3aecb3b2f71bc6842ee460a87bd07018f530", 65536),
    "payload_65k": ("48358e5b8a37c0af11fd5568d68f5fae5d3edcb3be21ba6c7d3515d4ecb7186d", 66560),
    "repeat_63k": ("6a95277fe915a852df57f872d9f9c0863777626dfd68d9e418242fc26973dbd0", 64512),
    "repeat_64k": ("9b839dd63b8ce0258e03f87b1c8c3aecb3b2f71bc6842ee460a87bd07018f530", 65536),
    "repeat_65k": ("48358e5b8a37c0af11fd5568d68f5fae5d3edcb3be21ba6c7d3515d4ecb7186d", 66560),
    "rand_block_gap": ("902e8412f2eb660d653e1577b614e396e62b6aaa8a8189df164899ec2be5b8d7", 48192),
    "zeros_100k": ("9192c25b734fcbadbe32dadc28089c60db0e39f90cc20ce2e5733f57261acc0c", 100000),
}
# crafted vectors: hex input, windowBits, expected result
CRAFTED = [
    ("len285_fixed", "4b1c451f0000", -16,
     {"ret": 1, "total_in": 6, "total_out": 1004,
      "sha256": "e49ae8cdb99d3a579bdd73690f5868cf892f3bb56f126eba6a88888b1f232afc"}),
    ("d64_empty_dist_reject", "05c081080000000020d6fd250e01", -16,
     {"ret": -3, "msg": "invalid distances set", "total_in": 13, "total_out": 0}),
    ("d64_empty_dist_std", "05c081080000000020d6fd250e01", -15,
     {"ret": 1, "total_in": 14, "total_out": 3, "sha256": hashlib.sha256(b"aaa").hexdigest()}),
    ("empty_fixed_trailing", "03000000", -15, {"ret": 1, "total_in": 2, "total_out": 0}),
    ("empty_stored_d64", "010000ffff", -16, {"ret": 1, "total_in": 5, "total_out": 0}),
    ("empty_input", "", -15, {"ret": -5, "total_in": 0, "total_out": 0}),
]
# error known-answers on fixtures
FIXTURE_ERRORS = [
    ("payload_64k", -15, None, {"ret": -3, "msg": "too many length or distance symbols", "total_in": 4475, "total_out": 61151}),
    ("10k_lines", -15, ("truncate", 6261), {"ret": -5, "msg": None, "total_in": 6261, "total_out": 59435}),
    ("10k_lines", 31, None, {"ret": -3, "msg": "incorrect header check", "total_in": 2, "total_out": 0}),
    ("payload_64k", -16, ("xor", 2000, 0xff), {"ret": 1, "msg": None, "total_in": 4531, "total_out": 65784}),
]
# sha256(trace text)[:16] of the JS/C-ABI call schedule
TRACES = [
    ("100k_lines", -16, 4096, 38, "63e6ef87f588bb01"),
    ("zeros_100k", -16, 4096, 3, "072f9e562121f38e"),
    ("10k_lines", -15, 1000, 14, "fc36175a7188b7a5"),
    ("10k_lines", -16, 32768, 3, "4b63070d6fc89ee8"),
]


def fixture(name):
    with open(os.path.join(HERE, "ref-data", name + ".deflate64"), "rb") as f:
        return f.read()


def mutate(data, how):
    if how is None:
        return data
    if how[0] == "truncate":
        return data[:how[1]]
    b = bytearray(data)
    b[how[1]] ^= how[2]
    return bytes(b)


def main():
    man = {"fixtures": {}, "crafted": [], "fixture_errors": [], "traces": []}
    for name, (sha, n) in SURVEY_OUT.items():
        out, info = O.oneshot(fixture(name), -16)
        got = hashlib.sha256(out).hexdigest()
        assert (got, len(out), info["ret"]) == (sha, n, 1), name
        man["fixtures"][name] = {"sha256": sha, "len": n, "total_in": info["total_in"], "wbits": -16}
    for name, hx, wb, exp in CRAFTED:
        out, info = O.oneshot(bytes.fromhex(hx), wb)
        for k, v in exp.items():
            got = hashlib.sha256(out).hexdigest() if k == "sha256" else info[k]
            assert got == v, (name, k, got, v)
        man["crafted"].append({"name": name, "hex": hx, "wbits": wb, "expect": exp})
    for name, wb, how, exp in FIXTURE_ERRORS:
        out, info = O.oneshot(mutate(fixture(name), how), wb)
        for k, v in exp.items():
            assert info[k] == v, (name, k, info[k], v)
        man["fixture_errors"].append({"fixture": name, "wbits": wb, "mutate": how, "expect": exp})
    for name, wb, w, calls, h in TRACES:
        tr, _ = O.js_schedule(fixture(name), w, wb)
        assert tr.count("\n") == calls and hashlib.sha256(tr.encode()).hexdigest()[:16] == h, name
        man["traces"].append({"fixture": name, "wbits": wb, "write": w, "calls": calls, "sha256_16": h})
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print("manifest ok")


if __name__ == "__main__":
    main()
