#!/usr/bin/env python3
"""Every BASELINE.json GPU configuration on one MI355X, plus the host-inclusive
(PCIe) rate — the numbers DESIGN.md §Measurements quotes.  bench.py stays the
driver's single headline line (north star); this is the wider table.

    python tools/bench_configs.py [--only ns,ipv4,tcp64,mixed,bimodal,jumbo,jumbo_all,host,router,ns64k,hostpatch,wrap,streams,batchv,stack] [--iters 20]

Batches that fit the 256 MiB Infinity Cache (ipv4 98 MB, tcp64 67 MB) are
rotated over >= 4 distinct copies (>= 393 / 268 MB) so every launch reads HBM.
Times are HIP events on the launch stream around `iters` back-to-back launches
(median of 5 rounds); the `streams` rows issue a stream of short batches
(configs 2, 3) on two HIP streams in turn, so one batch's drain overlaps the
next one's ramp; the `batchv` rows hand K = 8 such batches to ONE call
(ics_ipv4_tcp_batchv / ics_checksum_batchv: one launch, one stream) and
report the time per batch.  GiB = 2^30 B of algorithmic bytes (segment bytes, each
read once); metadata (inits, offsets, outputs) is reported separately.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from tcpip_network_protocol_stack_amd.engine import Engine, mixed_offsets  # noqa: E402

PEAK = 8000.0


def timed(fn, iters, rounds=5, settle_ms=150.0):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()  # settle power management (see bench.py --settle-ms)
    while (time.perf_counter() - t0) * 1e3 < settle_ms:
        for i in range(8):
            fn(i)
        torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for i in range(iters):
            fn(i)
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / 1e3 / iters)
    return statistics.median(ts)


def timed_streams(fn, iters, k, rounds=5):
    """Per-batch seconds of `iters` batches issued on k streams in turn:
    fn(i, stream, slot); first event to the last stream's end, median of
    `rounds` after one settling round."""
    main = torch.cuda.current_stream()
    streams = [torch.cuda.Stream(main.device) for _ in range(k)]
    ts = []
    for r in range(rounds + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(main)
        for s in streams:
            s.wait_stream(main)
        for i in range(iters):
            fn(i, streams[i % k], i % k)
        for s in streams:
            main.wait_stream(s)
        b.record(main)
        torch.cuda.synchronize()
        if r:
            ts.append(a.elapsed_time(b) / 1e3 / iters)
    return statistics.median(ts)


def emit(name, nbytes, t, meta_bytes=0, **kw):
    gbs = nbytes / t / 1e9
    print(json.dumps({"config": name, "bytes": nbytes, "us": round(t * 1e6, 2),
                      "GiB_s": round(nbytes / t / 2**30, 1), "GB_s": round(gbs, 1),
                      "frac_hbm_peak": round(gbs / PEAK, 4), "metadata_bytes": meta_bytes, **kw}), flush=True)


def rx_batch(eng, n, ack_frac, seed):
    """n raw IPv4/TCP datagrams back to back (packed offsets): a share
    ack_frac of 40-byte pure ACKs, the rest 1500-byte data segments, header
    fields set and both checksums PATCHed valid on the device"""
    rng = np.random.default_rng(seed)
    lens = np.where(rng.random(n) < ack_frac, 40, 1500).astype(np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]) + 16, dtype=np.uint8)
    s = off[:-1].astype(np.int64)
    buf[s], buf[s + 1] = 0x45, 0
    buf[s + 2], buf[s + 3] = (lens >> 8).astype(np.uint8), (lens & 255).astype(np.uint8)
    buf[s + 6], buf[s + 7], buf[s + 8], buf[s + 9] = 0x40, 0, 64, 6
    buf[s + 32] = 0x50  # TCP data offset 5
    d = torch.from_numpy(buf).cuda()
    doff = torch.from_numpy(off.view(np.int64)).cuda()
    eng.ipv4_tcp_batch(d, 2, n=n, offsets=doff)  # PATCH: valid checksums
    return d, doff, int(off[-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="ns,ipv4,tcp64,mixed,bimodal,jumbo,jumbo_all,host,streams")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", default="compute,patch,verify", help="ipv4 rows: which ics_ipv4_tcp_batch modes")
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed warm-up per row (0 for counter passes, which serialise every dispatch)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--warm-server", type=int, default=-1,
                    help="stack rows: a second engine with its tick server resident (idle limit in us; 0: the "
                         "second engine without a server, the control) poked before every row")
    ap.add_argument("--wrap-device-only", action="store_true", help="wrap rows: skip the host-memory rows")
    args = ap.parse_args()
    global timed
    _timed = timed
    timed = lambda fn, iters, **kw: _timed(fn, iters, **{"rounds": args.rounds,  # noqa: E731
                                                          "settle_ms": args.settle_ms, **kw})
    only = set(args.only.split(","))
    eng = Engine(0)
    eng_nobin = Engine(0)
    eng_nobin.set_binning(0)  # ICS_BINNING_SINGLE: single-geometry dispatch of offsets batches, for comparison
    os.environ["ICSUM_FORCE"] = "bin=1"
    eng_nocache = Engine(0)  # binned on every call: the binning passes without the plan cache
    del os.environ["ICSUM_FORCE"]
    dev = torch.device("cuda", 0)

    if "ns" in only:  # north star: 1 M x 1500 B, pseudo-header inits
        n, L, seed = 1 << 20, 1500, 0x10710000
        d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed)
        init = eng.pseudo_inits(n, seed, seg_len=L)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        t = timed(lambda i=0: eng.checksum_batch(d, n=n, stride=L, seg_len=L, init=init, out=out), args.iters)
        emit("ns_1Mx1500", n * L, t, n * 6, entry="ics_checksum_batch")
        del d

    if "ipv4" in only:  # config 2: 64 Ki x 1500 B IPv4 datagrams, fused header+pseudo+TCP
        n, L, seed, R = 1 << 16, 1500, 0x10710002, 6
        bufs = []
        for r in range(R):
            d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
            eng.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
            bufs.append(d)
        ip = torch.empty(n, dtype=torch.int16, device=dev)
        tcp = torch.empty(n, dtype=torch.int16, device=dev)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        if "patch" not in args.modes.split(","):  # VERIFY rows need valid checksum fields
            for d in bufs:
                eng.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)
        for mode, nm in ((0, "compute"), (2, "patch"), (1, "verify")):
            if nm not in args.modes.split(","):
                continue
            t = timed(lambda i=0: eng.ipv4_tcp_batch(bufs[i % R], mode, n=n, stride=L, dgram_len=L,
                                                     ip_ck=ip, tcp_ck=tcp, status=st), args.iters * 3)
            emit(f"ipv4_64Kix1500_{nm}", n * L, t, n * 5, entry="ics_ipv4_tcp_batch", rotation=R)
        assert (st.cpu().numpy() == 0x0F).all()
        del bufs

    if "router" in only:  # router TTL batch (ttl-- + header checksum) over 1 M x 1500 B
        # Each call forwards a datagram once (TTL 64 -> 63 ...), so the batch
        # cannot be re-run for the usual 150 ms settle: the chip is settled on
        # the NS workload instead, then 6 rotating copies (63 forwards each)
        # take 5 rounds of `iters` calls; every datagram must still forward.
        n, L, seed, R = 1 << 20, 1500, 0x10710003, 6
        bufs = []
        for r in range(R):
            d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
            eng.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
            eng.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)  # PATCH: valid header checksums
            bufs.append(d)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        warm = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed)
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) < 0.15:
            for _ in range(8):
                eng.checksum_batch(warm, n=n, stride=L, seg_len=L)
            torch.cuda.synchronize()
        del warm
        iters = min(args.iters, (63 * R - R) // 5)
        for i in range(R):
            eng.router_ttl_batch(bufs[i], n=n, stride=L, dgram_len=L, status=st)
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(iters):
                eng.router_ttl_batch(bufs[i % R], n=n, stride=L, dgram_len=L, status=st)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / 1e3 / iters)
        assert (st.cpu().numpy() == 1).all(), "router batch stopped forwarding"
        t = statistics.median(ts)
        # the same step with the forwarded headers apart (read-only batch, 20 B per datagram to one array)
        hd = torch.empty(n * 20, dtype=torch.uint8, device=dev)
        th = timed(lambda i=0: eng.router_ttl_headers(bufs[i % R], n=n, stride=L, dgram_len=L, hdrs=hd, status=st),
                   args.iters)
        assert (st.cpu().numpy() == 1).all()
        print(json.dumps({"config": "router_ttl_headers_1Mx1500", "datagrams": n, "us": round(th * 1e6, 2),
                          "Mdgram_s": round(n / th / 1e6, 1), "header_GB_s": round(n * 40 / th / 1e9, 1),
                          "line_GB_s": round(n * 128 / th / 1e9, 1),
                          "frac_hbm_peak_lines": round(n * 128 / th / 1e9 / PEAK, 4),
                          "entry": "ics_router_ttl_headers", "rotation": R,
                          "note": "20 header bytes read + 20 written per datagram; payloads untouched"}), flush=True)
        # algorithmic: 20 header bytes read + 4 written per datagram; the
        # memory system moves at least one 128-B line per datagram
        print(json.dumps({"config": "router_ttl_1Mx1500", "datagrams": n, "us": round(t * 1e6, 2),
                          "Mdgram_s": round(n / t / 1e6, 1), "header_GB_s": round(n * 24 / t / 1e9, 1),
                          "line_GB_s": round(n * 128 / t / 1e9, 1),
                          "frac_hbm_peak_lines": round(n * 128 / t / 1e9 / PEAK, 4),
                          "entry": "ics_router_ttl_batch", "rotation": R}), flush=True)
        del bufs

    if "hostpatch" in only:  # PATCH from host memory (the transmit side): 256 Ki x 1500 B IPv4/TCP datagrams
        n, L, seed = 1 << 18, 1500, 0x10710002
        d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed)
        eng.ipv4_tcp_headers(d, n, L, L, seed)
        src = d.cpu().numpy()
        del d
        for pinned in (True, False):
            h = torch.empty(n * L, dtype=torch.uint8, pin_memory=pinned).numpy()
            h[:] = src
            eng.ipv4_tcp_batch_host(h, n, 2, stride=L, dgram_len=L)  # warm (staging allocated)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                _, _, st = eng.ipv4_tcp_batch_host(h, n, 2, stride=L, dgram_len=L)
                ts.append(time.perf_counter() - t0)
            assert (st == 0x0F).all()
            emit(f"host_patch_256Kix1500_{'pinned' if pinned else 'pageable'}", n * L, statistics.median(ts),
                 n * 5, entry="ics_ipv4_tcp_batch_host(PATCH)")

    if "ns64k" in only:  # reference point for config 2: plain checksum over the same 64 Ki x 1500 B, rotated
        n, L, seed, R = 1 << 16, 1500, 0x10710002, 6
        ds = [eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
              for r in range(R)]
        out = torch.empty(n, dtype=torch.int16, device=dev)
        t = timed(lambda i=0: eng.checksum_batch(ds[i % R], n=n, stride=L, seg_len=L, out=out), args.iters * 3)
        emit("plain_64Kix1500", n * L, t, n * 2, entry="ics_checksum_batch", rotation=R)
        del ds

    if "streams" in only:  # a stream of short batches on two HIP streams in turn (configs 2, 3)
        K = 2
        n, L, seed, R = 1 << 16, 1500, 0x10710002, 6
        bufs = []
        for r in range(R):
            d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
            eng.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
            eng.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)
            bufs.append(d)
        outs = [(torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
                 torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(K)]
        for mode, nm in ((0, "compute"), (2, "patch"), (1, "verify")):
            t = timed_streams(lambda i, s, j: eng.ipv4_tcp_batch(bufs[i % R], mode, n=n, stride=L, dgram_len=L,
                                                                ip_ck=outs[j][0], tcp_ck=outs[j][1],
                                                                status=outs[j][2], stream=s), args.iters * 3, K)
            emit(f"ipv4_64Kix1500_{nm}_2streams", n * L, t, n * 5, entry="ics_ipv4_tcp_batch", rotation=R, streams=K)
        assert all((o[2].cpu().numpy() == 0x0F).all() for o in outs)
        t = timed_streams(lambda i, s, j: eng.checksum_batch(bufs[i % R], n=n, stride=L, seg_len=L, out=outs[j][0],
                                                            stream=s), args.iters * 3, K)
        emit("plain_64Kix1500_2streams", n * L, t, n * 2, entry="ics_checksum_batch", rotation=R, streams=K)
        del bufs
        n, L, seed = 1 << 20, 64, 0x10710003
        ds = [eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
              for r in range(R)]
        inits = [eng.pseudo_inits(n, seed, seg_len=L, index0=r * n) for r in range(R)]
        o16 = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(K)]
        t = timed_streams(lambda i, s, j: eng.checksum_batch(ds[i % R], n=n, stride=L, seg_len=L, init=inits[i % R],
                                                            out=o16[j], stream=s), args.iters * 3, K)
        emit("tcp_1Mx64_2streams", n * L, t, n * 6, entry="ics_checksum_batch", rotation=R, streams=K)
        del ds

    if "batchv" in only:  # K = 8 short batches in ONE call on one stream (configs 2, 3)
        K = 8
        n, L, seed = 1 << 16, 1500, 0x10710002
        bufs = []
        for r in range(2 * K):  # two sets of K: every call reads 786 MB, beyond the 256 MiB Infinity Cache
            d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
            eng.ipv4_tcp_headers(d, n, L, L, seed, index0=r * n)
            eng.ipv4_tcp_batch(d, 2, n=n, stride=L, dgram_len=L)
            bufs.append(d)
        outs = [dict(ip_ck=torch.empty(n, dtype=torch.int16, device=dev),
                     tcp_ck=torch.empty(n, dtype=torch.int16, device=dev),
                     status=torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(K)]
        sets = [[dict(dgrams=bufs[s * K + j], n=n, stride=L, dgram_len=L, **outs[j]) for j in range(K)]
                for s in range(2)]
        for mode, nm in ((0, "compute"), (2, "patch"), (1, "verify")):
            t = timed(lambda i=0: eng.ipv4_tcp_batchv(sets[i % 2], mode), args.iters)
            emit(f"ipv4_64Kix1500_{nm}_batchv{K}", n * L, t / K, n * 5, entry="ics_ipv4_tcp_batchv",
                 batches_per_call=K, note="time per batch")
        assert all((o["status"].cpu().numpy() == 0x0F).all() for o in outs)
        o16 = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(K)]
        psets = [[dict(data=bufs[s * K + j], n=n, stride=L, seg_len=L, out=o16[j]) for j in range(K)]
                 for s in range(2)]
        t = timed(lambda i=0: eng.checksum_batchv(psets[i % 2]), args.iters)
        emit(f"plain_64Kix1500_batchv{K}", n * L, t / K, n * 2, entry="ics_checksum_batchv", batches_per_call=K,
             note="time per batch")
        del bufs, sets, psets
        n, L, seed = 1 << 20, 64, 0x10710003
        ds = [eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
              for r in range(2 * K)]
        inits = [eng.pseudo_inits(n, seed, seg_len=L, index0=r * n) for r in range(2 * K)]
        sets = [[dict(data=ds[s * K + j], n=n, stride=L, seg_len=L, init=inits[s * K + j], out=torch.empty(n, dtype=torch.int16, device=dev))
                 for j in range(K)] for s in range(2)]
        t = timed(lambda i=0: eng.checksum_batchv(sets[i % 2]), args.iters)
        emit(f"tcp_1Mx64_batchv{K}", n * L, t / K, n * 6, entry="ics_checksum_batchv", batches_per_call=K,
             note="time per batch")
        del ds, sets

    if "tcp64" in only:  # config 3: 1 M x 64 B TCP segments with pseudo inits
        n, L, seed, R = 1 << 20, 64, 0x10710003, 6
        ds = [eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L)
              for r in range(R)]
        inits = [eng.pseudo_inits(n, seed, seg_len=L, index0=r * n) for r in range(R)]
        out = torch.empty(n, dtype=torch.int16, device=dev)
        t = timed(lambda i=0: eng.checksum_batch(ds[i % R], n=n, stride=L, seg_len=L, init=inits[i % R], out=out),
                  args.iters * 3)
        emit("tcp_1Mx64", n * L, t, n * 6, entry="ics_checksum_batch", rotation=R)
        del ds

    if "mixed" in only:  # config 4: 1 M mixed 64 B - 64 KiB, packed offsets (odd starts)
        n, seed = 1 << 20, 0x10710004
        off = mixed_offsets(n, seed)
        d = eng.fill_bytes(torch.empty(int(off[-1]), dtype=torch.uint8, device=dev), seed)
        doff = torch.from_numpy(off.view(np.int64)).to(dev)
        init = eng.pseudo_inits(n, seed, offsets=doff)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        for tag, e in (("", eng), ("_unbinned", eng_nobin), ("_auto_nocache", eng_nocache)):
            t = timed(lambda i=0: e.checksum_batch(d, offsets=doff, init=init, out=out), args.iters // 2 or 1)
            emit("mixed_1M_64B_64KiB" + tag, int(off[-1]), t, n * 14, entry="ics_checksum_batch(offsets)",
                 dispatch={"": "auto (default, plan cache)", "_unbinned": "single launch",
                           "_auto_nocache": "auto, binning passes every call"}[tag])
        del d

    if "bimodal" in only:  # ACK-sized and MSS-sized TCP segments interleaved, packed offsets
        n, seed = 2 << 20, 0x10710006
        rng = np.random.default_rng(seed)
        lens = np.where(rng.random(n) < 0.5, 40, 1460) + rng.integers(0, 4, n)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum(lens)
        d = eng.fill_bytes(torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device=dev), seed)
        doff = torch.from_numpy(off.view(np.int64)).to(dev)
        init = eng.pseudo_inits(n, seed, offsets=doff)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        for tag, e in (("", eng), ("_unbinned", eng_nobin), ("_auto_nocache", eng_nocache)):
            t = timed(lambda i=0: e.checksum_batch(d, offsets=doff, init=init, out=out), args.iters)
            emit("bimodal_2M_40B_1460B" + tag, int(off[-1]), t, n * 14, entry="ics_checksum_batch(offsets)",
                 dispatch={"": "auto (default, plan cache)", "_unbinned": "single launch",
                           "_auto_nocache": "auto, binning passes every call"}[tag])
        del d

    if "rxmix" in only:  # received traffic: raw IPv4/TCP datagrams, ACKs among MTU segments, valid headers
        n = 1 << 20
        ip = torch.empty(n, dtype=torch.int16, device=dev)
        tcp = torch.empty(n, dtype=torch.int16, device=dev)
        stt = torch.empty(n, dtype=torch.uint8, device=dev)
        for af in (0.25, 0.5, 0.75):
            d, doff, nbytes = rx_batch(eng, n, af, 11)
            t = timed(lambda i=0: eng.ipv4_tcp_batch(d, 1, n=n, offsets=doff, ip_ck=ip, tcp_ck=tcp, status=stt),
                      args.iters)
            info = eng.dispatch_info()
            emit(f"rxmix_1M_{int(af * 100)}pct_acks_verify", nbytes, t, n * 13, entry="ics_ipv4_tcp_batch VERIFY",
                 last_kernel=info["kernel"], datagrams_per_wave=info["unroll"])
            del d

    if "jumbo" in only:  # config 5 per-GPU shard (weak scaling unit): 1 M x 9000 B
        n, L, seed = 1 << 20, 9000, 0x10710005
        d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed)
        init = eng.pseudo_inits(n, seed, seg_len=L)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        t = timed(lambda i=0: eng.checksum_batch(d, n=n, stride=L, seg_len=L, init=init, out=out), args.iters // 2)
        emit("jumbo_1Mx9000_shard", n * L, t, n * 6, entry="ics_checksum_batch")
        del d

    if "jumbo_all" in only:  # config 5 whole batch on ONE GPU (strong-scaling N=1 point): 8 M x 9000 B
        n, L, seed = 8 << 20, 9000, 0x10710005
        d = eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed)
        init = eng.pseudo_inits(n, seed, seg_len=L)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        t = timed(lambda i=0: eng.checksum_batch(d, n=n, stride=L, seg_len=L, init=init, out=out), 3, rounds=3)
        emit("jumbo_8Mx9000_1gpu", n * L, t, n * 6, entry="ics_checksum_batch")
        del d
        torch.cuda.empty_cache()

    if "host" in only:  # PCIe-inclusive: host bytes in, host u16 out (ics_checksum_batch_host)
        from oracle import oracle as orc  # workload bytes only (spec generator)

        n, L, seed = 1 << 18, 1500, 0x10710000
        for pinned in (True, False):
            h = torch.empty(n * L, dtype=torch.uint8, pin_memory=pinned)
            h.numpy()[:] = orc.fill_bytes(seed, 0, n * L)
            hi = np.array([orc.pseudo_init(seed, i, L) for i in range(n)], dtype=np.uint32)
            eng.checksum_batch_host(h.numpy(), n, stride=L, seg_len=L, init=hi)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                eng.checksum_batch_host(h.numpy(), n, stride=L, seg_len=L, init=hi)
                ts.append(time.perf_counter() - t0)
            emit(f"host_inclusive_256Kix1500_{'pinned' if pinned else 'pageable'}", n * L, statistics.median(ts),
                 n * 6, entry="ics_checksum_batch_host", note="H2D + kernel + D2H, 3-slot pipeline")
            if pinned:  # the link's own ceiling: one plain H2D copy of the same pinned bytes, no kernel
                d = torch.empty(n * L, dtype=torch.uint8, device=dev)
                d.copy_(h, non_blocking=True)
                torch.cuda.synchronize()
                ts = []
                for _ in range(5):
                    t0 = time.perf_counter()
                    d.copy_(h, non_blocking=True)
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                emit("pcie_h2d_copy_256Kix1500_pinned", n * L, statistics.median(ts), 0, entry="torch copy_ (hipMemcpyAsync)",
                     note="reference ceiling for the host-inclusive rows: H2D only")
                del d
    if "wrap" in only:  # device-side wrap_tcp_in_ip (headers + both checksums written)
        from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE

        # the stack's segments: MSS 1000 B payload (TCPConfig::MAX_PAYLOAD_SIZE) -> 1040-byte datagrams
        n, L, seed, R = 1 << 20, 1040, 0x10710006, 2
        rng = np.random.default_rng(6)
        m = np.zeros(n, dtype=TCP_MSG_DTYPE)
        for f, hi in (("src", 2**32), ("dst", 2**32), ("seqno", 2**32), ("ackno", 2**32), ("src_port", 2**16),
                      ("dst_port", 2**16), ("window", 2**16)):
            m[f] = rng.integers(0, hi, n, dtype=np.uint64)
        m["flags"], m["ttl"] = 0x10, 128
        dm = torch.from_numpy(m.view(np.uint8).copy()).to(dev)
        ds = [eng.fill_bytes(torch.empty(n * L, dtype=torch.uint8, device=dev), seed, pos0=r * n * L) for r in range(R)]
        t = timed(lambda i=0: eng.tcp_wrap_batch(ds[i % R], dm, n=n, stride=L, dgram_len=L), args.iters)
        emit("wrap_1Mx1040_device", n * L, t, n * 28, entry="ics_tcp_wrap_batch", rotation=R,
             note="bytes = datagram bytes (payload read once, 40 header bytes written per datagram)")
        del ds
        # headers kept apart (iovec form): payload-only batch, 40-byte headers to one coalesced array
        P = L - 40
        ps = [eng.fill_bytes(torch.empty(n * P, dtype=torch.uint8, device=dev), seed, pos0=r * n * P) for r in range(R)]
        hd = torch.empty(n * 40, dtype=torch.uint8, device=dev)
        t = timed(lambda i=0: eng.tcp_wrap_headers(ps[i % R], dm, hd, n=n, stride=P, payload_len=P), args.iters)
        emit("wrap_headers_apart_1Mx1000_device", n * (P + 40), t, n * 28, entry="ics_tcp_wrap_headers",
             rotation=R, note="bytes = datagram bytes (1000-byte payloads read, 40-byte headers written coalesced)")
        out = torch.empty(n, dtype=torch.int16, device=dev)
        t = timed(lambda i=0: eng.checksum_batch(ps[i % R], n=n, stride=P, seg_len=P, out=out), args.iters)
        emit("plain_1Mx1000_reference_point", n * P, t, n * 2, entry="ics_checksum_batch", rotation=R,
             note="the same payload batch through the plain checksum kernel (no headers, no records)")
        del ps
        nh = 1 << 18
        for pinned in (() if args.wrap_device_only else (True, False)):
            h = torch.empty(nh * L, dtype=torch.uint8, pin_memory=pinned).numpy()
            h[:] = 7
            eng.tcp_wrap_batch_host(h, m[:nh], nh, stride=L, dgram_len=L)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                eng.tcp_wrap_batch_host(h, m[:nh], nh, stride=L, dgram_len=L)
                ts.append(time.perf_counter() - t0)
            emit(f"wrap_host_256Kix1040_{'pinned' if pinned else 'pageable'}", nh * L, statistics.median(ts), nh * 68,
                 entry="ics_tcp_wrap_batch_host", note="H2D payloads + kernel + D2H of the 40 header bytes")

    if "stack" in only:  # one stack tick: transmit wrap and receive VERIFY on their own buffers, interleaved
        # (with one plan-cache entry each call evicted the other's plan; the keyed slots must
        # leave each call's time and launch exactly what it is when the call runs alone)
        from tcpip_network_protocol_stack_amd.engine import TCP_MSG_DTYPE

        n, seed = 1 << 18, 0x10710007
        rng = np.random.default_rng(seed)
        # received: half pure ACKs (40 B), half MTU segments, back to back, with
        # valid IPv4/TCP headers (ver 4, hlen 5, len, DF, ttl 64, TCP, data
        # offset 5; both checksums set by a PATCH pass) — what a TUN read ring holds
        rl = np.where(rng.random(n) < 0.5, 40, 1500)
        roff = np.zeros(n + 1, dtype=np.uint64)
        roff[1:] = np.cumsum(rl)
        rbuf = rng.integers(0, 256, int(roff[-1]) + 16, dtype=np.uint8)
        rs = roff[:-1].astype(np.int64)
        rbuf[rs], rbuf[rs + 1], rbuf[rs + 2], rbuf[rs + 3] = 0x45, 0, (rl >> 8).astype(np.uint8), (rl & 255).astype(np.uint8)
        rbuf[rs + 6], rbuf[rs + 7], rbuf[rs + 8], rbuf[rs + 9], rbuf[rs + 32] = 0x40, 0, 64, 6, 0x50
        # transmitted: payloads of 0..1000 bytes (TCPConfig::MAX_PAYLOAD_SIZE) behind 40 bytes of room
        pl = rng.integers(0, 1001, n)
        tl = 40 + pl
        toff = np.zeros(n + 1, dtype=np.uint64)
        toff[1:] = np.cumsum(tl)
        poff = np.zeros(n + 1, dtype=np.uint64)  # the same payloads alone (headers apart)
        poff[1:] = np.cumsum(pl)
        rx = torch.from_numpy(rbuf).to(dev)
        tx = eng.fill_bytes(torch.empty(int(toff[-1]) + 16, dtype=torch.uint8, device=dev), seed + 1)
        px = eng.fill_bytes(torch.empty(int(poff[-1]) + 16, dtype=torch.uint8, device=dev), seed + 2)
        hd = torch.empty(n * 40, dtype=torch.uint8, device=dev)
        drof = torch.from_numpy(roff.view(np.int64)).to(dev)
        dtof = torch.from_numpy(toff.view(np.int64)).to(dev)
        dpof = torch.from_numpy(poff.view(np.int64)).to(dev)
        eng.ipv4_tcp_batch(rx, 2, n=n, offsets=drof)  # PATCH: valid checksums
        m = np.zeros(n, dtype=TCP_MSG_DTYPE)
        for f, hi in (("src", 2**32), ("dst", 2**32), ("seqno", 2**32), ("ackno", 2**32), ("src_port", 2**16),
                      ("dst_port", 2**16), ("window", 2**16)):
            m[f] = rng.integers(0, hi, n, dtype=np.uint64)
        m["flags"], m["ttl"] = 0x10, 128
        dm = torch.from_numpy(m.view(np.uint8).copy()).to(dev)
        ip = torch.empty(n, dtype=torch.int16, device=dev)
        tcp = torch.empty(n, dtype=torch.int16, device=dev)
        stt = torch.empty(n, dtype=torch.uint8, device=dev)

        def verify():
            eng.ipv4_tcp_batch(rx, 1, n=n, offsets=drof, ip_ck=ip, tcp_ck=tcp, status=stt)

        def wrap():
            eng.tcp_wrap_batch(tx, dm, n=n, offsets=dtof)

        def wrap_apart():  # the iovec form: payload arena + the 40-byte headers in an array of their own
            eng.tcp_wrap_headers(px, dm, hd, n=n, offsets=dpof)

        def per_call(fn, other, calls):
            """median of per-call HIP-event times of fn, each call alone or right after `other`"""
            st = torch.cuda.current_stream()
            evs = []
            for _ in range(calls):
                if other:
                    other()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(st)
                fn()
                b.record(st)
                evs.append((a, b))
            torch.cuda.synchronize()
            return statistics.median(a.elapsed_time(b) / 1e3 for a, b in evs), eng.dispatch_info()

        for _ in range(4):  # every key misses once, then its plan lands
            verify()
            wrap()
            wrap_apart()
        torch.cuda.synchronize()
        calls = args.iters * args.rounds
        rows = {}
        poke = lambda: None  # noqa: E731
        if args.warm_server >= 0:  # does a resident block elsewhere on the card change the idle-queue cost?
            warm = Engine(0)
            warm.set_tick_server(args.warm_server)
            wbuf = torch.zeros(64, dtype=torch.uint8, pin_memory=True).numpy()

            def poke():
                warm.checksum_batch_host(wbuf, 1, stride=64, seg_len=64)
                print(json.dumps({"warm_server_us": args.warm_server, "kernel": warm.dispatch_info()["kernel"]}),
                      file=sys.stderr)
        entries = {verify: "ics_ipv4_tcp_batch VERIFY", wrap: "ics_tcp_wrap_batch",
                   wrap_apart: "ics_tcp_wrap_headers"}
        for name, fn, other in (("verify_alone", verify, None), ("verify_after_wrap", verify, wrap),
                                ("wrap_alone", wrap, None), ("wrap_after_verify", wrap, verify),
                                ("wrap_apart_alone", wrap_apart, None), ("wrap_apart_after_verify", wrap_apart, verify)):
            poke()
            before = eng.dispatch_info()
            t, info = per_call(fn, other, calls)
            rows[name] = t
            nbytes = int(roff[-1]) if fn is verify else int(toff[-1])  # wrap: payloads + 40 header bytes each
            emit(f"stack_tick_{name}", nbytes, t, n * (5 if fn is verify else 28),
                 entry=entries[fn],
                 last_kernel=info["kernel"], last_plan=info["plan"],
                 plan_hits=info["plan_hits"] - before["plan_hits"],
                 plan_misses=info["plan_misses"] - before["plan_misses"],
                 note="median per-call HIP-event time; 256 Ki datagrams, packed offsets")
        # the same calls back to back (events around `iters` calls): no host
        # gap between a call's first event and its launch
        for name, fn in (("verify_b2b", verify), ("wrap_b2b", wrap), ("wrap_apart_b2b", wrap_apart)):
            poke()
            t = timed(lambda i=0, f=fn: f(), args.iters)
            nbytes = int(roff[-1]) if fn is verify else int(toff[-1])
            emit(f"stack_tick_{name}", nbytes, t, n * (5 if fn is verify else 28),
                 entry=entries[fn],
                 note="back-to-back calls, events around the run; 256 Ki datagrams, packed offsets")
        # one whole tick: the receive VERIFY and the transmit headers-apart wrap,
        # on one stream in turn, and on two streams (forked from and joined
        # back into the caller's stream every tick: the results of both are
        # needed before the next tick, util/tcp_minnow_socket/tcp_minnow_socket.h:138-164)
        s1, s2 = torch.cuda.current_stream(), torch.cuda.Stream(device=dev)
        fork, join = torch.cuda.Event(), torch.cuda.Event()

        def tick_one(i=0):
            verify()
            wrap_apart()

        def tick_two(i=0):
            fork.record(s1)
            s2.wait_event(fork)
            eng.tcp_wrap_headers(px, dm, hd, n=n, offsets=dpof, stream=s2)
            verify()
            join.record(s2)
            s1.wait_event(join)

        both = int(roff[-1]) + int(toff[-1])
        for name, fn in (("both_one_stream", tick_one), ("both_two_streams", tick_two)):
            poke()
            t = timed(fn, args.iters)
            emit(f"stack_tick_{name}", both, t, n * 33,
                 entry="ics_ipv4_tcp_batch VERIFY + ics_tcp_wrap_headers",
                 note="one tick per step: 256 Ki received datagrams VERIFYed and 256 Ki transmitted datagrams "
                      "wrapped with the headers apart, back to back, events around the run")
        assert (stt.cpu().numpy() == 0x0F).all(), "the receive batch must verify"
        del rx, tx, px
    eng.close()


if __name__ == "__main__":
    main()
