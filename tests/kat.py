"""Helpers to expand tests/golden/kat.json vectors."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
KIND = {"received": 1, "close": 2, "ping": 3, "pong": 4}


def load():
    with open(os.path.join(HERE, "golden", "kat.json")) as f:
        return json.load(f)


def payload_of(v):
    if "pattern" in v:
        kind, n = v["pattern"].split(":")
        n = int(n)
        if kind == "zeros":
            return bytes(n)
        if kind == "ramp":
            return bytes(i & 0xFF for i in range(n))
        raise ValueError(kind)
    return bytes.fromhex(v.get("payload", ""))


def key_of(v):
    b = bytes.fromhex(v["key"])
    return b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24


def events_of(v):
    return [(KIND[k], bytes.fromhex(p), s) for k, p, s in v["events"]]
