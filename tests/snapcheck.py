"""Python counterparts of the reference test helpers (test_common.go).

read_snapshot_file  test_common.go:149-193
assert_equal        test_common.go:222-285 (order compared per destination only)
check_tokens        test_common.go:298-328 (token conservation)
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEST_DATA = os.path.join(ROOT, "tests", "golden", "test_data")


def scenarios():
    with open(os.path.join(ROOT, "tests", "golden", "scenarios.json")) as f:
        return json.load(f)["tests"]


def read_text(name):
    with open(os.path.join(TEST_DATA, name)) as f:
        return f.read()


def read_snapshot_file(name):
    sid, tokens, msgs = 0, {}, []
    for line in read_text(name).split("\n"):
        if not line or line.startswith("#"):
            continue
        parts = line.split()
        if len(parts) == 1:
            sid = int(line)
        elif len(parts) == 2:
            tokens[parts[0]] = int(parts[1])
        elif len(parts) == 3:
            if "token" not in parts[2]:
                raise ValueError("Unknown message: " + parts[2])
            nums = re.findall(r"[0-9]+", parts[2])
            if len(nums) != 1:
                raise ValueError("Unable to parse token message: " + parts[2])
            msgs.append((parts[0], parts[1], int(nums[0])))
    return sid, tokens, msgs


def _per_dest(msgs):
    out = {}
    for m in msgs:
        out.setdefault(m[1], []).append(tuple(m))
    return out


def assert_equal(expected, actual):
    """expected/actual: (id, tokens dict, [(src, dest, amount)])."""
    eid, etok, emsg = expected
    aid, atok, amsg = actual
    assert eid == aid, f"Snapshot IDs do not match: {eid} != {aid}"
    assert len(etok) == len(atok), f"Snapshot {eid}: Number of tokens do not match"
    assert len(emsg) == len(amsg), f"Snapshot {eid}: Number of messages do not match: {emsg} vs {amsg}"
    for k, v in etok.items():
        assert atok.get(k) == v, f"Snapshot {eid}: Tokens on {k} do not match: {etok} vs {atok}"
    assert _per_dest(emsg) == _per_dest(amsg), f"Snapshot {eid}: messages differ: {emsg} vs {amsg}"


def check_tokens(final_tokens, snapshots):
    expected = sum(final_tokens.values())
    for sid, tok, msgs in snapshots:
        got = sum(tok.values()) + sum(m[2] for m in msgs)
        assert got == expected, f"Snapshot {sid}: simulator has {expected} tokens, snapshot has {got}"
