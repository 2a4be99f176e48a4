"""Shared fixture handling for the parity tests (inputs/expectations from tests/golden/)."""
import numpy as np

from conftest import golden


def kat_cases(tags=None):
    """checksum_kat.json cases as (init, [piece bytes], value); fill cases expanded."""
    out = []
    for c in golden("checksum_kat.json")["cases"]:
        if tags and c["tag"] not in tags:
            continue
        if c["tag"] == "fill":
            pieces = [bytes([c["fill"]]) * c["len"]]
        else:
            pieces = [bytes.fromhex(p) for p in c["pieces"]]
        out.append((c["init"], pieces, c["value"], c["tag"]))
    return out


def pack_contiguous(segs, lead=0):
    """Back-to-back segments (n+1 offsets), the first starting at `lead`."""
    offs = [lead]
    for s in segs:
        offs.append(offs[-1] + len(s))
    buf = np.frombuffer(b"\xa5" * lead + b"".join(segs) + b"\0" * 16, dtype=np.uint8).copy()
    return buf, np.array(offs, dtype=np.uint64)


def wires(name, tags=None):
    return [c for c in golden(name)["cases"] if tags is None or c.get("tag") in tags]
