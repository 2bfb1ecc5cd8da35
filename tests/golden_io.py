"""Loader for tests/golden/records.json (vectors captured from the reference
tlslite by tests/golden/make_golden.py).  Regenerates large plaintexts from
their `pt_gen` seed with the same SHA-256 counter stream."""
import hashlib
import json
import os

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "records.json")


def gen_bytes(seed, n):
    out = bytearray()
    ctr = 0
    while len(out) < n:
        out += hashlib.sha256(seed.encode() + ctr.to_bytes(4, "big")).digest()
        ctr += 1
    return bytes(out[:n])


def rec_pt(rec):
    if "pt" in rec:
        return bytes.fromhex(rec["pt"])
    return gen_bytes(rec["pt_gen"], rec["pt_len"])


def case_data(case):
    if "pt" in case:
        return bytes.fromhex(case["pt"])
    return gen_bytes(case["pt_gen"], case["pt_len"])


def wire_matches(entry, wire):
    wire = bytes(wire)
    if "wire" in entry:
        return wire == bytes.fromhex(entry["wire"])
    return (len(wire) == entry["wire_len"] and hashlib.sha256(wire).hexdigest() == entry["wire_sha256"])


def case_keys(case):
    return (bytes.fromhex(case["key"]), bytes.fromhex(case["iv"]), bytes.fromhex(case["mac_key"]),
            bytes.fromhex(case["fixed_iv"]) if case["fixed_iv"] else None, case["seq"])


_cache = None


def load_golden():
    global _cache
    if _cache is None:
        with open(PATH) as f:
            _cache = json.load(f)["cases"]
    return _cache


def load_json(name):
    """Another committed fixture under tests/golden/ (sessions.json, batches.json, ...)."""
    with open(os.path.join(os.path.dirname(PATH), name)) as f:
        return json.load(f)
