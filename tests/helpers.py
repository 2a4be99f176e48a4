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


# ---- configs.json "6": the full-size wrap spec (oracle/ref/golden_gen.cpp config_wrap)
def wrap6_records(fields, dtype):
    """n x 32 spec bytes -> ics_tcp_msg records (numpy, `dtype` =
    engine.TCP_MSG_DTYPE): src, dst, seqno, ackno big-endian u32; ports and
    window big-endian u16; flag byte 1 FIN, 2 SYN, 4 RST, 0x10 ACK present
    (ackno 0 without it); ttl 128, id 0 as wrap_tcp_in_ip sets them."""
    f = np.asarray(fields, dtype=np.uint8).reshape(-1, 32).astype(np.uint64)
    be32 = lambda k: (f[:, k] << 24) | (f[:, k + 1] << 16) | (f[:, k + 2] << 8) | f[:, k + 3]  # noqa: E731
    be16 = lambda k: (f[:, k] << 8) | f[:, k + 1]  # noqa: E731
    m = np.zeros(len(f), dtype=dtype)
    m["src"], m["dst"], m["seqno"] = be32(0), be32(4), be32(8)
    flags = f[:, 22] & 0x17
    m["ackno"] = np.where(flags & 0x10, be32(12), 0)
    m["src_port"], m["dst_port"], m["window"] = be16(16), be16(18), be16(20)
    m["flags"], m["ttl"], m["id"] = flags, 128, 0
    return m


def oracle_wrap_wire(orc, payload, r):
    """serialize(wrap_tcp_in_ip(msg)) by the oracle: the header fields as
    serialize() lays them out, both checksums by its PATCH
    (ipv4_header.cpp:113-123, tcp_segment.cpp:109-118)."""
    L = (40 + len(payload)) & 0xFFFF
    b = bytearray([0x45, 0, L >> 8, L & 255, int(r["id"]) >> 8, int(r["id"]) & 255, 0x40, 0, int(r["ttl"]), 6, 0, 0])
    b += int(r["src"]).to_bytes(4, "big") + int(r["dst"]).to_bytes(4, "big")
    b += int(r["src_port"]).to_bytes(2, "big") + int(r["dst_port"]).to_bytes(2, "big")
    b += int(r["seqno"]).to_bytes(4, "big") + int(r["ackno"]).to_bytes(4, "big")
    b += bytes([0x50, int(r["flags"])]) + int(r["window"]).to_bytes(2, "big") + b"\0\0\0\0" + bytes(payload)
    _, _, st, w = orc.ipv4_tcp(bytes(b), 2)
    assert st & 0x03 == 0x03
    return w


# ---- tests/golden/endtoend_capture.npz (oracle/make_endtoend_capture.py)
def endtoend_capture():
    """The frames the unmodified reference stack exchanged in BASELINE config
    1 (128 KiB transfer), as captured on the relay: (frames uint8 buffer,
    frame offsets n+1, direction, offsets n_ip+1 of the IPv4 datagrams inside
    the frames — each starts 14 bytes into its EthernetFrame, so the starts
    are unaligned exactly as a receive arena of frames holds them)."""
    import os

    z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "endtoend_capture.npz"),
                allow_pickle=False)
    frames, off, direction = z["frames"], z["offsets"].astype(np.uint64), z["direction"]
    ip = [i for i in range(len(off) - 1) if frames[off[i] + 12] == 0x08 and frames[off[i] + 13] == 0x00]
    # IPv4 datagram k = [its frame's start + 14, the frame's end)
    starts = np.array([off[i] + 14 for i in ip], dtype=np.uint64)
    ends = np.array([off[i + 1] for i in ip], dtype=np.uint64)
    buf = np.concatenate([frames, np.zeros(16, dtype=np.uint8)])
    return buf, off, direction, starts, ends


def ip_packed(buf, starts, ends, lead=0):
    """The captured IPv4 datagrams back to back (the IP layer's receive arena)."""
    segs = [buf[int(s):int(e)].tobytes() for s, e in zip(starts, ends)]
    return pack_contiguous(segs, lead)
