"""GPU: one engine context shared by several host threads, each on its own
HIP stream — INTEGRATION.md §5: "One context may serve several streams at
once".  ctypes releases the GIL for the call, so the threads' calls overlap
inside the library and touch its shared state together:

* the device scratch lease (binned dispatch of an offsets batch above the
  binning threshold, the two-pass wrap's payload sums): a call on another
  stream must wait for the previous user's kernels, and growth must wait too;
* the plan cache: more batch keys than slots, so slots are re-keyed (LRU)
  while plan kernels queued by other threads for the old key are still in
  flight — their words carry the old generation and must not be trusted;
* the multi-batch grouping and the diagnostics counters;
* round 4: the router step with its headers apart and a variable-length
  batch that reaches the tile launch from its cached plan.

Every thread's outputs after every round (each round starts from sentinel
outputs) must equal what the same calls gave one at a time on one stream.
The serial results themselves are checked against the oracle (the binned
batch in full, IPv4 and wrap on samples; full parity of each call is the
other test modules' job).  Bar: bit-exact.

Power check (round 3, once, not kept): with the scratch lease's cross-stream
wait removed from icsum_ctx.h, this test failed in its first two rounds
(threads 0 and 1, the binned batch's outputs)."""
import threading

import numpy as np
import pytest

from test_gpu_parity import _random_datagrams, _t

pytestmark = pytest.mark.gpu

THREADS = 4
ROUNDS = 12


@pytest.fixture(scope="module")
def ceng():
    """Two-pass wrap for every batch size (the scratch user that small batches reach)."""
    from conftest import engine_with

    yield from engine_with({"wrap_passes": 2})


def _offsets(lens, lead=0):
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    return off + lead


class Job:
    """One thread's inputs (its own device buffers: its own plan-cache keys),
    its output tensors and the calls that fill them."""

    def __init__(self, eng, rng, dgram_bytes, dgram_off, wrap_pay, wrap_msgs):
        import torch

        self.eng = eng
        # binned + plan-cached offsets batch (n above the 64 Ki binning threshold)
        lens = rng.choice([0, 1, 40, 64, 577, 1500, 3000, 9000], 70000)
        self.off1 = _offsets(lens, lead=3)
        self.buf1 = rng.integers(0, 256, int(self.off1[-1]) + 16, dtype=np.uint8)
        self.d_buf1, self.d_off1 = _t(self.buf1), _t(self.off1)
        self.init1 = rng.integers(0, 2**32, 70000, dtype=np.uint32)
        self.d_init1 = _t(self.init1)
        # IPv4 VERIFY over raw datagrams (plan-cached geometry from 16 Ki datagrams up)
        self.d_dg, self.d_dgoff = _t(dgram_bytes), _t(dgram_off)
        self.ndg = len(dgram_off) - 1
        # device wrap, headers apart, two passes (scratch for the payload sums)
        self.nw = len(wrap_msgs)
        self.d_pay, self.d_msgs = _t(wrap_pay), _t(wrap_msgs.view(np.uint8))
        # multi-batch call: a 1500-byte fixed-stride batch, config 3's dense shape, an offsets batch
        self.bv_bufs = [_t(rng.integers(0, 256, 3000 * 1500 + 16, dtype=np.uint8)),
                        _t(rng.integers(0, 256, 5000 * 64, dtype=np.uint8))]
        self.bv_init = _t(rng.integers(0, 2**32, 5000, dtype=np.uint32))
        off3 = _offsets(rng.integers(0, 2000, 2000), lead=1)
        self.bv_off = _t(off3)
        self.bv_buf3 = _t(rng.integers(0, 256, int(off3[-1]) + 16, dtype=np.uint8))
        # a variable-length batch above the tile threshold (the tile launch once its plan is cached)
        self.toff = _offsets(40 + rng.integers(0, 1001, 140_000), lead=2)
        self.tbuf = rng.integers(0, 256, int(self.toff[-1]) + 16, dtype=np.uint8)
        self.d_toff, self.d_tbuf = _t(self.toff), _t(self.tbuf)
        dev = "cuda:0"
        self.outs = [torch.empty(70000, dtype=torch.int16, device=dev),
                     torch.empty(self.ndg, dtype=torch.int16, device=dev),
                     torch.empty(self.ndg, dtype=torch.int16, device=dev),
                     torch.empty(self.ndg, dtype=torch.uint8, device=dev),
                     torch.empty(self.nw * 40, dtype=torch.uint8, device=dev),
                     torch.empty(self.nw, dtype=torch.int16, device=dev),
                     torch.empty(self.nw, dtype=torch.int16, device=dev),
                     torch.empty(3000, dtype=torch.int16, device=dev),
                     torch.empty(5000, dtype=torch.int16, device=dev),
                     torch.empty(2000, dtype=torch.int16, device=dev),
                     torch.empty(self.ndg * 20, dtype=torch.uint8, device=dev),  # router: forwarded headers
                     torch.empty(self.ndg, dtype=torch.uint8, device=dev),
                     torch.empty(140_000, dtype=torch.int16, device=dev)]
        self.want = None

    def reset(self, stream):
        import torch

        with torch.cuda.stream(stream):
            for t in self.outs:
                t.fill_(0x5A)

    def run(self, stream):
        e, o = self.eng, self.outs
        e.checksum_batch(self.d_buf1, offsets=self.d_off1, init=self.d_init1, out=o[0], stream=stream)
        e.ipv4_tcp_batch(self.d_dg, 1, n=self.ndg, offsets=self.d_dgoff, ip_ck=o[1], tcp_ck=o[2], status=o[3],
                         stream=stream)
        e.tcp_wrap_headers(self.d_pay, self.d_msgs, o[4], n=self.nw, stride=100, payload_len=100, ip_ck=o[5],
                           tcp_ck=o[6], stream=stream)
        e.checksum_batchv([dict(data=self.bv_bufs[0], n=3000, stride=1500, seg_len=1500, out=o[7]),
                           dict(data=self.bv_bufs[1], n=5000, stride=64, seg_len=64, init=self.bv_init, out=o[8]),
                           dict(data=self.bv_buf3, n=2000, offsets=self.bv_off, out=o[9])], stream=stream)
        e.router_ttl_headers(self.d_dg, n=self.ndg, offsets=self.d_dgoff, hdrs=o[10], status=o[11], stream=stream)
        e.checksum_batch(self.d_tbuf, offsets=self.d_toff, out=o[12], stream=stream)


def test_one_context_many_threads_and_streams(ceng, orc):
    import torch
    from test_gpu_wrap import _oracle_wire, _random_batch

    rng = np.random.default_rng(0xC0C0)
    segs = _random_datagrams(rng, 20000)
    dgram_off = _offsets([len(s) for s in segs], lead=5)
    dgram_bytes = np.frombuffer(b"\0" * 5 + b"".join(segs) + b"\0" * 16, dtype=np.uint8).copy()
    _, wmsgs = _random_batch(rng, 5000, fixed=100)
    wrap_pay = rng.integers(0, 256, 5000 * 100, dtype=np.uint8)
    jobs = [Job(ceng, rng, dgram_bytes, dgram_off, wrap_pay, wmsgs) for _ in range(THREADS)]

    # serial results, each call alone on the default stream (twice: the
    # second call of a key runs its cached plan)
    s0 = torch.cuda.current_stream()
    for j in jobs:
        for _ in range(2):
            j.reset(s0)
            j.run(s0)
        torch.cuda.synchronize()
        j.want = [t.clone() for t in j.outs]
    # ... spot-checked against the oracle
    j = jobs[0]
    got = j.want[0].cpu().numpy().view(np.uint16)
    assert np.array_equal(got, orc.checksum_batch(j.buf1, 70000, offsets=j.off1, init=j.init1))
    ip, tcp, st = (j.want[k].cpu().numpy() for k in (1, 2, 3))
    for i in range(0, 20000, 487):
        wip, wtcp, wst, _ = orc.ipv4_tcp(segs[i], 1)
        assert (int(ip.view(np.uint16)[i]), int(tcp.view(np.uint16)[i]), int(st[i])) == (wip, wtcp, wst), i
    assert np.array_equal(j.want[12].cpu().numpy().view(np.uint16), orc.checksum_batch(j.tbuf, 140_000, offsets=j.toff))
    hd = j.want[4].cpu().numpy()
    for i in range(0, 5000, 311):
        want = _oracle_wire(orc, [b"\0" * 40 + wrap_pay[100 * i:100 * i + 100].tobytes()], wmsgs[i:i + 1])[0]
        assert hd[40 * i:40 * i + 40].tobytes() == want[:40], i

    before = ceng.dispatch_info()
    errors = []
    start = threading.Barrier(THREADS)

    def body(job, tid):
        try:
            s = torch.cuda.Stream(device=0)
            start.wait(timeout=60)
            for r in range(ROUNDS):
                job.reset(s)
                job.run(s)
                s.synchronize()
                for k, (g, w) in enumerate(zip(job.outs, job.want)):
                    if not torch.equal(g, w):
                        errors.append(f"thread {tid} round {r} output {k} differs")
                        return
        except Exception as exc:  # surfaced by the assert below
            errors.append(f"thread {tid}: {exc!r}")

    threads = [threading.Thread(target=body, args=(j, t)) for t, j in enumerate(jobs)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in threads), "a worker thread did not finish"
    assert not errors, errors
    after = ceng.dispatch_info()
    # 8 plannable keys over 4 slots: the cache was consulted on every call
    lookups = (after["plan_hits"] + after["plan_misses"]) - (before["plan_hits"] + before["plan_misses"])
    assert lookups >= THREADS * ROUNDS * 2, (before, after)
