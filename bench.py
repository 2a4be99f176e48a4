#!/usr/bin/env python3
"""Device-resident Internet-checksum throughput (BASELINE.json metric).

One "step" = one ics_checksum_batch pass (InternetChecksum{pseudo}.add(seg).value(),
util/tools/checksum.h:17-41 with the TCP pseudo-header seed of
util/ipv4_header/ipv4_header.cpp:103-110) over one resident batch.  At N=1 the
workload is the north-star configuration: 1 M x 1500 B segments (1.57 GB, far
larger than the 256 MiB Infinity Cache, so every step streams from HBM).
At N>1 (torchrun, one process per GPU) every rank owns its own 1 M-segment
shard of one global spec stream — weak scaling, no data-path collective; the
only collectives are the timing barrier and the max-over-ranks reduction, both
over gloo on the host (the device is synchronised before each, so nothing on
the path needs RCCL — north_star: "no RCCL collective").

The same line carries `config5`: BASELINE config 5 (8 M x 9000 B, 75.5 GB)
sharded over the N GPUs — strong scaling, its own timed region after the NS
one — so a 1/2/4/8 run measures both the north-star weak-scaling value and the
config-5 curve.

Every timed leg checks its own outputs against the reference's digests
(tests/golden/configs.json, made by the reference's InternetChecksum,
util/tools/checksum.h:20-41): `bit_exact` = EVERY rank's NS shard against
the reference's digest of that shard (`configs.json["0"].shard_sha256[r]`,
global segments [r 2^20, (r+1) 2^20) of config 0's spec stream; shard 0 is the
config-0 batch) and `config5.bit_exact` = all ranks' config-5 outputs gathered
over gloo (the whole 8 M-segment batch).  `per_rank` lists each rank's device
(PCI address and UUID), kernel time, wall time, rate, output digest and its
match, so an N > 1 line can be read rank by rank; `ranks_per_gpu` counts the
ranks per distinct device id gathered, not a device count.

`--gpus N` without an outer launcher starts the N ranks itself (one process
per GPU via torch.distributed.run on 127.0.0.1; this parent never touches the
GPU); under a launcher, WORLD_SIZE must equal --gpus.

Prints ONE JSON line (rank 0) with `roofline` (HIP-event kernel time vs the
8 TB/s HBM peak; PMC traffic from a rocprofv3 child pass) and `cpu_baseline`
(the reference's own InternetChecksum, compiled from /root/reference into
oracle/_ref/, over the same bytes — the whole NS batch — on every CPU this
process may use, outputs compared with the GPU's).  At N=1 it also carries
`host_inclusive` (north_star: the path starts and ends in host memory): the
same NS batch through ics_checksum_batch_host from page-locked memory (H2D,
kernel and D2H pipelined; GB/s, outputs compared with the device run's), and
the per-call latency of a per-tick host batch of 1 and 16 segments (one
zero-copy launch and a completion word; ctypes call, preallocated outputs).
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident GiB/s, Internet checksum over segment batch, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md §Chip-level parameters)
KERNEL_PREFIX = "k_checksum"

# reference digests (tests/golden/configs.json, computed by the reference's own
# InternetChecksum, util/tools/checksum.h:20-41): a weak-scaling workload's
# rank r checks its shard (global segments [r n, (r+1) n) of the spec stream)
# against shard_sha256[r] where the config has them ("0": ranks 0-7), else
# rank 0 against out_sha256 (its shard IS the BASELINE batch) and the other
# ranks stay unchecked (bit_exact None, not False); a strong workload gathered
# over the ranks is the whole batch
GOLDEN_KEY = {"ns_1Mx1500": "0", "tcp_1Mx64": "3", "jumbo_8Mx9000": "5"}

WORKLOADS = {
    # name: (segments, segment bytes, seed, scaling) — DESIGN.md §Workload spec.
    # "weak": `segments` per rank (the global batch grows with N);
    # "strong": `segments` in total, sharded across the N ranks.
    "ns_1Mx1500": (1 << 20, 1500, 0x10710000, "weak"),
    "tcp_1Mx64": (1 << 20, 64, 0x10710003, "weak"),
    "jumbo_1Mx9000": (1 << 20, 9000, 0x10710005, "weak"),
    "jumbo_8Mx9000": (8 << 20, 9000, 0x10710005, "strong"),  # BASELINE config 5
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="ns_1Mx1500", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline budget (0 = skip)")
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="minimum untimed warm-up (ms of back-to-back launches) after --warmup")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC child pass")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = every CPU this process may run on)")
    ap.add_argument("--launch-check", action="store_true",
                    help="ranks report their rank/world wiring over gloo and exit (no GPU use)")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip the BASELINE config-5 strong-scaling sub-measurement")
    ap.add_argument("--config5-steps", type=int, default=0, help="timed steps of config 5 (0 = --steps)")
    ap.add_argument("--no-host", action="store_true", help="skip the host_inclusive sub-object")
    return ap.parse_args()


# ------------------------------------------------------------ rank launcher -
def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` without an outer launcher: start N ranks, one process per GPU,
    through torch.distributed.run on 127.0.0.1.  This parent never touches the
    GPU (nothing here imports torch), and the ranks are children, not an exec."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    return subprocess.call(cmd, env=env)


def golden_configs():
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        return json.load(f)


def u16_host(t):
    import numpy as np

    return t.cpu().numpy().view(np.uint16)


def sha256_u16(a):
    import hashlib

    import numpy as np

    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def gather_u16(out, dist):
    """The ranks' u16 outputs in rank order, concatenated on rank 0 (None on
    the others): one gloo gather of host copies, after the timed region."""
    import numpy as np

    mine = u16_host(out)
    if dist is None:
        return mine
    parts = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object(mine.tobytes(), parts, dst=0)
    if parts is None:
        return None
    return np.frombuffer(b"".join(parts), dtype=np.uint16)


def gather_rows(row, dist):
    """Every rank's row (a dict) on rank 0, in rank order (None elsewhere)."""
    if dist is None:
        return [row]
    rows = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object(row, rows, dst=0)
    return rows


def init_gloo(dist):
    """Join the gloo group.  Gloo prints "[Gloo] Rank r is connected to ..."
    on fd 1 while the group forms; that goes to stderr, so stdout holds only
    rank 0's one JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo")
        dist.barrier()
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def launch_check(rank, world):
    """Every rank joins a gloo group and rank 0 prints what each one saw."""
    import torch.distributed as dist

    init_gloo(dist)
    seen = [None] * world
    dist.all_gather_object(seen, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "-1")),
                                  "world_size": dist.get_world_size(),
                                  "master_addr": os.environ.get("MASTER_ADDR"), "pid": os.getpid()})
    if rank == 0:
        print(json.dumps({"launch_check": seen}), flush=True)
    dist.destroy_process_group()


# ------------------------------------------------------------ PMC traffic --
def pmc_traffic(args):
    """HBM bytes per launch of the checksum kernel from FETCH_SIZE, in a child
    `rocprofv3 --pmc FETCH_SIZE` run of this same workload (its own pass, no
    tracing domains).  gfx950: FETCH_SIZE (KiB) reads 1/2 of a wide coalesced
    stream (MI355X_MICROARCH.md §HBM), so bytes = 2 * 1024 * FETCH_SIZE."""
    rocprof = shutil.which("rocprofv3")
    if not rocprof:
        return None, "rocprofv3 not found"
    out = tempfile.mkdtemp(prefix="icsum_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = [rocprof, "--pmc", "FETCH_SIZE", "--output-format", "csv", "-d", out, "-o", "pmc", "--",
           sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "3", "--warmup", "1",
           "--workload", args.workload, "--cpu-seconds", "0", "--no-pmc"]
    # a one-rank child on this rank's GPU, also when this process is a rank
    # of an N > 1 run (it runs before the rank joins its group)
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "MASTER_ADDR",
                        "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["LOCAL_RANK"] = os.environ.get("LOCAL_RANK", "0")
    try:
        subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                       cwd=out, env=env)
        rows = []
        for f in glob.glob(os.path.join(out, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                rows += [r for r in csv.DictReader(fh) if KERNEL_PREFIX in r.get("Kernel_Name", "")]
        vals = [float(r["Counter_Value"]) for r in rows if r.get("Counter_Name") == "FETCH_SIZE"]
        if not vals:
            return None, "no FETCH_SIZE rows"
        vals = vals[1:] if len(vals) > 1 else vals  # drop the first (cold) launch
        return 2.0 * 1024.0 * sum(vals) / len(vals), "rocprofv3 --pmc FETCH_SIZE x2 (gfx950 correction)"
    except Exception as e:  # reported, never fatal
        return None, f"pmc pass failed: {type(e).__name__}"
    finally:
        shutil.rmtree(out, ignore_errors=True)


# ------------------------------------------------------------ CPU baseline -
def cpu_share():
    """(threads, how) — every CPU this process may run on: its affinity mask,
    capped by a cgroup CPU quota when one is set (on the GPU box the machine
    shows all its CPUs while one GPU's job gets a share of them)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    how = f"affinity {n} of {os.cpu_count()} host CPUs"
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                quota, period = f.read().split()[:2]
            if quota != "max":
                q = max(1, int(int(quota) // int(period)))
                if q < n:
                    n, how = q, f"cgroup quota {quota}/{period} = {q} CPUs ({how})"
        except (OSError, ValueError):
            pass
    return n, how


def cpu_baseline(data_d, init_d, out_d, seg, budget_s, threads=0):
    """The reference's own InternetChecksum (oracle/_ref, compiled from
    /root/reference) — or the oracle port when that build is absent — over the
    whole batch of this run (its first 2 GiB for the larger workloads) (the same bytes and inits, copied back from HBM),
    on every CPU this process may use, repeated until ~budget_s; its outputs
    are compared with the GPU's for every segment.  Plus a 1-core figure."""
    import numpy as np

    from oracle import oracle as orc

    n = min(init_d.numel(), (2 << 30) // seg)  # the whole batch up to 2 GiB (NS: all 1.47 GiB)
    data = data_d[: n * seg].cpu().numpy()
    init = init_d[:n].cpu().numpy().view(np.uint32)
    gpu = out_d[:n].cpu().numpy().view(np.uint16)
    out = np.empty(n, dtype=np.uint16)
    share, how = cpu_share()
    threads = threads or share
    ref = orc.ref_lib()
    kind = "reference" if ref is not None else "port"

    def one(count, nthreads):
        if ref is not None:
            ref.ref_checksum_batch(data.ctypes.data, None, seg, seg, init.ctypes.data, out.ctypes.data,
                                   count, nthreads)
        else:
            out[:count] = orc.checksum_batch(data[: count * seg], count, stride=seg, seg_len=seg,
                                             init=init[:count], threads=nthreads)

    def timed(nthreads, budget, count):
        """passes of `count` segments on `nthreads` threads until `budget` s"""
        passes, t0 = 0, time.perf_counter()
        while True:
            one(count, nthreads)
            passes += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return passes, el

    one(n, threads)  # warm, and the full-batch comparison
    match = bool((out == gpu).all())
    passes, el = timed(threads, 0.8 * budget_s, n)
    gib = passes * n * seg / el / 2**30
    one_n = max(1, min(n, (256 << 20) // seg))  # 1 core: a 256 MiB prefix
    p1, el1 = timed(1, 0.2 * budget_s, one_n)
    gib1 = p1 * one_n * seg / el1 / 2**30
    return {"value": round(gib, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "value_1core": round(gib1, 3), "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "cores_basis": how,
            "sample": f"{'the whole batch' if n == init_d.numel() else 'a prefix of the batch'} ({n} segments x {seg} B = {n * seg / 2**30:.2f} GiB), {passes} passes "
                      f"in {el:.1f} s on {threads} threads; 1 core: first {one_n} segments, {p1} passes "
                      f"in {el1:.1f} s; all {n} outputs bit-identical to the GPU's: {match}"}


def host_inclusive(eng, data, init, out, n, seg, passes=3, calls=300):
    """The PCIe-inclusive rate of the same batch and the latency of per-tick
    host calls ("Host-inclusive" and "Per-tick host batches")."""
    import numpy as np
    import torch

    h = torch.empty(data.numel(), dtype=torch.uint8, pin_memory=True)
    h.copy_(data)
    hn = h.numpy()
    hi = init.cpu().numpy()
    want = out.cpu().numpy().view(np.uint16)
    got = eng.checksum_batch_host(hn, n, stride=seg, seg_len=seg, init=hi)  # staging set up before the clock
    same = bool((got == want).all())
    t0 = time.perf_counter()
    for _ in range(passes):
        eng.checksum_batch_host(hn, n, stride=seg, seg_len=seg, init=hi)
    el = time.perf_counter() - t0
    tick = {}
    res = np.empty(16, dtype=np.uint16)
    fn, ctx = eng.lib.ics_checksum_batch_host, eng.ctx
    a_in, a_init, a_res = hn.ctypes.data, hi.ctypes.data, res.ctypes.data  # a caller's buffers: addresses known
    for k in (1, 16):
        ts = []
        for c in range(calls + 20):
            t1 = time.perf_counter()
            rc = fn(ctx, a_in, None, seg, seg, a_init, a_res, k)
            if c >= 20:
                ts.append(time.perf_counter() - t1)
            if rc:
                raise RuntimeError(f"ics_checksum_batch_host: {rc}")
        same = same and bool((res[:k] == want[:k]).all())
        tick[f"segments_{k}_us"] = round(sorted(ts)[len(ts) // 2] * 1e6, 2)
    del h
    return {"entry": "ics_checksum_batch_host", "memory": "page-locked", "bytes": n * seg, "passes": passes,
            "GB_s": round(n * seg * passes / el / 1e9, 2), "outputs_equal_device": same,
            "tick_p50": tick, "tick_note": f"{seg}-byte segments, {calls} ctypes calls, preallocated outputs, buffer addresses taken once",
            "tick_p50_cpp": tick_cpp_guarded(calls),
            "tick_p50_cpp_server": tick_cpp_guarded(calls, "tick_server=20000"),
            "tick_p50_cpp_server_vram": tick_cpp_guarded(calls, "tick_server=20000,srv_vram=1"),
            "tick_cpp_note": "the same calls from C++ (tools/probe/tick_latency, dlopen of the in-tree libicsum.so, "
                             "1500-byte segments with inits, page-locked), no interpreter in the loop; _server: "
                             "with the resident tick server (ics_set_tick_server, 20 ms idle; 4 blocks, 16 segments each), "
                             "no launch per call; _server_vram: the same with its descriptors and each tick's bytes "
                             "written into device memory through the BAR (ICSUM_FORCE srv_vram, opt-in)"}


def tick_cpp(calls, force=None):
    """p50 of per-tick ics_checksum_batch_host calls timed in C++ (a child
    process: the interpreter's ctypes overhead is not in these numbers);
    force: the context's ICSUM_FORCE (e.g. the resident tick server)"""
    exe = os.path.join(ROOT, "tools", "probe", "tick_latency")
    lib = os.path.join(ROOT, "tcpip_network_protocol_stack_amd", "libicsum.so") + (f"@{force}" if force else "")
    if not os.path.exists(exe):
        return None
    env = dict(os.environ, TICK_OPS="checksum", TICK_SIZES="1,16,64", TICK_MEM="pinned", TICK_CALLS=str(calls))
    r = subprocess.run([exe, lib], env=env, capture_output=True, text=True, timeout=120)
    if r.returncode:
        raise RuntimeError(f"tick_latency: {r.returncode} {r.stderr.strip()[-300:]}")
    out = {}
    for line in r.stdout.splitlines():
        d = json.loads(line)
        out[f"segments_{d['n']}_us"] = d["p50_us"]
    return out


def tick_cpp_guarded(calls, force=None):
    """tick_cpp, reported and never fatal (like pmc_traffic): a failure of
    this secondary figure must not cost the line its headline"""
    try:
        return tick_cpp(calls, force)
    except Exception as e:
        return {"error": f"{type(e).__name__}: {str(e)[-200:]}"}


def device_id(local):
    """(PCI address, UUID) of this rank's device: what identifies the card
    across processes, whatever the launcher's device visibility"""
    import torch

    p = torch.cuda.get_device_properties(local)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", str(getattr(p, "uuid", ""))


def ranks_per_gpu(rows):
    """The most ranks that shared one device, from the gathered device ids"""
    from collections import Counter

    return max(Counter((r["pci"], r["uuid"]) for r in rows).values())


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_cfg, seg, seed, scaling = WORKLOADS[args.workload]
    if args.launch_check:
        launch_check(rank, world)
        return

    # the PMC child pass runs before this process touches the GPU
    traffic, traffic_src = (None, "skipped")
    if not args.pmc_child and not args.no_pmc and rank == 0:
        # rank 0's launches (every rank runs the same per-GPU workload); at
        # N > 1 the other ranks wait in the group rendezvous meanwhile
        traffic, traffic_src = pmc_traffic(args)

    import torch

    from tcpip_network_protocol_stack_amd import shard
    from tcpip_network_protocol_stack_amd.engine import Engine

    # one process per GPU (ranks share a card when there are fewer GPUs than
    # ranks: the one-card rehearsal of an N-rank run)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        # host-side group for the timing barrier and the max over ranks only:
        # every rank synchronises its device before either, so a host
        # collective brackets exactly the same work an RCCL one would
        init_gloo(dist)
    eng = Engine(local)
    stream = torch.cuda.current_stream(dev)

    def timed(step, steps):
        """barrier + synchronize on both sides of `steps` back-to-back steps;
        returns (max-over-ranks wall seconds, this rank's HIP-event seconds per
        step on the launch stream)"""
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(stream)
        for _ in range(steps):
            step()
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        # this rank's time stops when its own steps have drained; the closing
        # barrier keeps the ranks bracketed, and the MAX makes the slowest
        # rank's time the job's (a barrier's own latency is not a step's work)
        elapsed = time.perf_counter() - t0
        if dist:
            dist.barrier()
        return shard.max_over_ranks(elapsed, dist), ev0.elapsed_time(ev1) / 1e3 / steps, elapsed

    def settle(step):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        # settle the chip's power management: a load step from idle leaves the
        # first ~10-50 ms of launches 5-25 % off steady state (measured, DESIGN.md
        # §Measurement); keep warming (untimed) until >= --settle-ms of kernels ran
        t_settle = time.perf_counter()
        while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
            for _ in range(8):
                step()
            torch.cuda.synchronize(dev)

    # rank r owns a contiguous range of global segments of ONE spec stream
    n_total = n_cfg * world if scaling == "weak" else n_cfg
    sh = shard.fixed_stride_shard(n_total, seg, seg, rank, world)
    n = sh.n
    data = torch.empty(sh.nbytes, dtype=torch.uint8, device=dev)
    eng.fill_bytes(data, seed, pos0=sh.byte0)
    init = eng.pseudo_inits(n, seed, seg_len=seg, index0=sh.index0)
    out = torch.empty(n, dtype=torch.int16, device=dev)

    def step():
        eng.checksum_batch(data, n=n, stride=seg, seg_len=seg, init=init, out=out, stream=stream)

    settle(step)
    if args.pmc_child:
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        return

    # kernel time: HIP events on the stream the kernel runs on, bracketing the
    # K back-to-back launches of the timed region (per-launch event pairs
    # would insert markers between dispatches and measure their gaps too)
    elapsed, kern_s, own_s = timed(step, args.steps)
    bytes_step = n * seg  # algorithmic bytes per rank per step (each byte read once)
    value = n_total * seg * args.steps / elapsed / 2**30  # all ranks' bytes / max-over-ranks time
    achieved = bytes_step / kern_s / 1e9  # GB/s, decimal like the 8 TB/s peak

    # the timed steps' outputs, checked against the reference's digests: rank
    # r's shard of a weak-scaling workload is global segments [r n, (r+1) n)
    # of one spec stream, and the reference's outputs for each such slice
    # are hashed in configs.json (shard 0 = the BASELINE batch itself)
    gold = golden_configs()
    ns_sha = sha256_u16(u16_host(out))
    key = GOLDEN_KEY.get(args.workload)
    # this rank's shard digest: global segments [rank n, (rank+1) n) of the
    # workload's spec stream (weak scaling: n per rank at any N)
    want = None
    if key and scaling == "weak":
        shards = gold[key].get("shard_sha256") or [gold[key]["out_sha256"]]
        want = shards[rank] if rank < len(shards) else None
    pci, uuid = device_id(local)
    per_rank = gather_rows({"rank": rank, "device": local, "pci": pci, "uuid": uuid, "segments": n,
                            "index0": sh.index0, "kernel_ms": round(kern_s * 1e3, 4),
                            "wall_ms_per_step": round(own_s / args.steps * 1e3, 4),
                            "GiB_s": round(bytes_step * args.steps / own_s / 2**30, 2),
                            "roofline_frac": round(achieved / HBM_PEAK_GBS, 4), "out_sha256": ns_sha,
                            "bit_exact": None if want is None else ns_sha == want}, dist)
    bit_exact, checked = None, "no reference digest for this workload"
    if key and scaling == "weak":
        if rank == 0:
            marks = [r["bit_exact"] for r in per_rank]
            unchecked = sum(m is None for m in marks)
            # a mismatch anywhere: False; every rank matched: True; some ranks
            # without a digest and no mismatch: None (partial, not a failure)
            bit_exact = False if any(m is False for m in marks) else (True if not unchecked else None)
            checked = (f"every rank's {n} outputs vs its reference shard digest "
                       f"(tests/golden/configs.json[{key!r}].shard_sha256[rank])"
                       + (f"; partial: {unchecked} rank(s) have no shard digest" if unchecked else ""))
    elif key:
        whole = gather_u16(out, dist)
        bit_exact = sha256_u16(whole) == gold[key]["out_sha256"] if rank == 0 else None
        checked = f"all ranks' {n_total} outputs vs tests/golden/configs.json[{key!r}].out_sha256"

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(data, init, out, seg, args.cpu_seconds, args.cpu_threads)
    host = None
    if rank == 0 and world == 1 and not args.no_host:
        host = host_inclusive(eng, data, init, out, n, seg)
    del data, init, out

    # BASELINE config 5: 8 M x 9000 B sharded over the N GPUs (strong scaling)
    config5 = None
    if not args.no_config5 and args.workload != "jumbo_8Mx9000":
        n5, seg5, seed5, _ = WORKLOADS["jumbo_8Mx9000"]
        sh5 = shard.fixed_stride_shard(n5, seg5, seg5, rank, world)
        torch.cuda.empty_cache()
        d5 = torch.empty(sh5.nbytes, dtype=torch.uint8, device=dev)
        eng.fill_bytes(d5, seed5, pos0=sh5.byte0)
        i5 = eng.pseudo_inits(sh5.n, seed5, seg_len=seg5, index0=sh5.index0)
        o5 = torch.empty(sh5.n, dtype=torch.int16, device=dev)

        def step5():
            eng.checksum_batch(d5, n=sh5.n, stride=seg5, seg_len=seg5, init=i5, out=o5, stream=stream)

        settle(step5)
        k5 = args.config5_steps or args.steps
        el5, kern5, own5 = timed(step5, k5)
        # the timed steps' outputs of every rank, gathered in rank order: the
        # whole 8 M-segment batch, against the reference's digest
        whole5 = gather_u16(o5, dist)
        rows5 = gather_rows({"rank": rank, "segments": sh5.n, "kernel_ms": round(kern5 * 1e3, 4),
                             "wall_ms_per_step": round(own5 / k5 * 1e3, 4),
                             "roofline_frac": round(sh5.n * seg5 / kern5 / 1e9 / HBM_PEAK_GBS, 4)}, dist)
        config5 = {"workload": "jumbo_8Mx9000", "scaling": "strong", "segments_total": n5,
                   "segments_per_gpu": sh5.n, "segment_bytes": seg5, "steps": k5,
                   "ms_per_step": round(el5 / k5 * 1e3, 4),
                   "value": round(n5 * seg5 * k5 / el5 / 2**30, 2), "unit": "GiB/s",
                   "kernel_ms": round(kern5 * 1e3, 4),
                   "roofline_frac": round(sh5.n * seg5 / kern5 / 1e9 / HBM_PEAK_GBS, 4),
                   "bit_exact": None if whole5 is None else sha256_u16(whole5) == gold["5"]["out_sha256"],
                   "checked": f"all ranks' {n5} outputs (gathered) vs tests/golden/configs.json['5'].out_sha256",
                   "per_rank": rows5}
        del d5, i5, o5
        torch.cuda.empty_cache()

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded splitmix64 spec, DESIGN.md §Workload spec)",
            "config": {"workload": args.workload, "segments_total": n_total, "segments_per_gpu": n,
                       "segment_bytes": seg,
                       "bytes_per_step_per_gpu": bytes_step, "inits": "IPv4 pseudo-header sums",
                       "entry": "ics_checksum_batch", "parallelism": f"shard{world}",
                       "ranks_per_gpu": ranks_per_gpu(per_rank),
                       "devices": len({(r["pci"], r["uuid"]) for r in per_rank})},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if traffic is None else round(traffic),
                         "kernel_ms": round(kern_s * 1e3, 4),
                         "traffic_source": traffic_src},
            "bit_exact": bit_exact,
            "checked": checked,
            "per_rank": per_rank,
            "cpu_baseline": cpu,
            "config5": config5,
            "host_inclusive": host,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
