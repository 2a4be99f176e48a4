#!/usr/bin/env python3
"""BASELINE config 1: the reference's apps/endtoend (two hosts, two routers,
frames relayed over UDP; /root/reference/apps/endtoend.cpp:240-408) moving
1 MiB of seeded bytes client -> server over 127.0.0.1, bit-exact.

The upstream relay (cs144.keithw.org) is replaced by a local UDP "bounce"
server: it learns the first two peers that say hello (endtoend sends three
empty datagrams first, endtoend.cpp:258-261) and forwards every non-empty
datagram from one to the other.

    python tools/endtoend_run.py BINARY [--bytes N] [--seed S] [--timeout T] [--capture FILE.npz]
                                 [--corrupt P]

prints one JSON line: ok (server stdout == client stdin), transfer_s (client start
until the server has written every byte), wall_s (both processes exited; includes the
TCP close linger of tcp_minnow_socket), bytes.

--capture keeps every frame the relay forwards (the serialized EthernetFrames
the two routers exchange, endtoend.cpp:118-124) in forwarding order: `frames`
(uint8, back to back), `offsets` (uint64, n + 1), `direction` (uint8: 0 from
the first peer — the server — to the second, 1 back), saved with numpy.

--corrupt P flips one random bit past the Ethernet header of a fraction P of
the IPv4 frames (seeded): the stack must drop each one at its checksum check
(a checksum failure is a loss) and TCP must retransmit, so the
transfer still arrives bit-exact; the line reports how many were flipped.
"""
import argparse
import json
import os
import selectors
import socket
import subprocess
import sys
import tempfile
import threading
import time


def seeded_bytes(n, seed):
    """splitmix64 stream (the workload spec of DESIGN.md §5), n bytes."""
    out = bytearray()
    c = 0
    while len(out) < n:
        z = (seed + (c + 1) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        z ^= z >> 31
        out += z.to_bytes(8, "little")
        c += 1
    return bytes(out[:n])


class Bounce(threading.Thread):
    """UDP relay between the first two distinct peers."""

    def __init__(self):
        super().__init__(daemon=True)
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.sock.bind(("127.0.0.1", 0))
        self.sock.setblocking(False)
        self.port = self.sock.getsockname()[1]
        self.peers = []
        self.forwarded = 0
        self.captured = []  # (direction, frame) when capturing
        self.capture = False
        self.corrupt = 0.0
        self.flipped = 0
        self.rng = None
        self.stop = threading.Event()

    def run(self):
        sel = selectors.DefaultSelector()
        sel.register(self.sock, selectors.EVENT_READ)
        while not self.stop.is_set():
            for _ in sel.select(timeout=0.05):
                while True:
                    try:
                        data, addr = self.sock.recvfrom(65536)
                    except BlockingIOError:
                        break
                    if addr not in self.peers and len(self.peers) < 2:
                        self.peers.append(addr)
                    if data and len(self.peers) == 2 and addr in self.peers:
                        other = self.peers[1 - self.peers.index(addr)]
                        if self.corrupt and len(data) > 14 and data[12:14] == b"\x08\x00" and \
                                self.rng.random() < self.corrupt:
                            b = bytearray(data)
                            bit = self.rng.randrange(8 * (len(b) - 14))
                            b[14 + bit // 8] ^= 1 << (bit % 8)
                            data = bytes(b)
                            self.flipped += 1
                        self.sock.sendto(data, other)
                        self.forwarded += 1
                        if self.capture:
                            self.captured.append((self.peers.index(addr), data))
        self.sock.close()


def run(binary, nbytes, seed, timeout, capture=None, corrupt=0.0):
    payload = seeded_bytes(nbytes, seed)
    bounce = Bounce()
    bounce.capture = capture is not None
    if corrupt:
        import random

        bounce.corrupt = corrupt
        bounce.rng = random.Random(seed)
    bounce.start()
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "client.in")
        with open(src, "wb") as f:
            f.write(payload)
        srv_out = os.path.join(td, "server.out")
        t0 = time.perf_counter()
        with open(os.devnull, "rb") as nul, open(srv_out, "wb") as so, open(src, "rb") as ci:
            server = subprocess.Popen([binary, "server", "127.0.0.1", str(bounce.port)], stdin=nul,
                                      stdout=so, stderr=subprocess.PIPE)
            time.sleep(0.2)  # the server says hello first, so the client's SYN is forwarded
            t_client = time.perf_counter()
            client = subprocess.Popen([binary, "client", "127.0.0.1", str(bounce.port)], stdin=ci,
                                      stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            t_data = None  # when the server's stdout holds every byte (before TCP's close linger)
            while t_data is None and time.perf_counter() - t0 < timeout and server.poll() is None:
                if os.path.getsize(srv_out) >= nbytes:
                    t_data = time.perf_counter() - t_client
                time.sleep(0.002)
            try:
                _, cerr = client.communicate(timeout=timeout)
                _, serr = server.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                client.kill()
                server.kill()
                client.communicate()
                server.communicate()
                bounce.stop.set()
                return {"ok": False, "error": "timeout", "binary": binary}
        wall = time.perf_counter() - t0
        with open(srv_out, "rb") as f:
            got = f.read()
    bounce.stop.set()
    bounce.join()
    if capture:
        import numpy as np

        frames = [f for _, f in bounce.captured]
        off = np.zeros(len(frames) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(f) for f in frames])
        np.savez(capture, frames=np.frombuffer(b"".join(frames), dtype=np.uint8), offsets=off,
                 direction=np.array([d for d, _ in bounce.captured], dtype=np.uint8))
    return {"ok": got == payload, "bytes": nbytes, "received": len(got),
            "transfer_s": None if t_data is None else round(t_data, 3), "wall_s": round(wall, 3),
            "frames_relayed": bounce.forwarded, "frames_corrupted": bounce.flipped, "client_rc": client.returncode, "server_rc": server.returncode,
            "binary": binary}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("binary")
    ap.add_argument("--bytes", type=int, default=1 << 20)
    ap.add_argument("--seed", type=int, default=0x10710001)
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--capture", default=None, help="save the relayed frames (.npz)")
    ap.add_argument("--corrupt", type=float, default=0.0, help="fraction of IPv4 frames with one bit flipped")
    a = ap.parse_args()
    r = run(a.binary, a.bytes, a.seed, a.timeout, a.capture, a.corrupt)
    print(json.dumps(r), flush=True)
    sys.exit(0 if r["ok"] else 1)


if __name__ == "__main__":
    main()
