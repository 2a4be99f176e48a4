"""GPU parity at byte bases of any address.

The reference sums bytes wherever they lie: InternetChecksum::add takes any
string_view (/root/reference/util/tools/checksum.h:20-28) and
IPv4Header::parse any buffer (util/ipv4_header/ipv4_header.cpp:9-59); a
receive arena of Ethernet frames holds its IPv4 datagrams 14 bytes in
(src/network_interface/network_interface.cpp:51).  So every batch call takes
d_bytes / d_dgrams / d_payloads at any address (include/icsum.h).  Here every
kernel family runs on batches whose base is 1, 2, 3, 8 or 14 bytes into a
fresh allocation (and 0 as the control), against the oracle on the same bytes:

  checksum   fixed stride and offsets through every lane-group shape (line
             grid, masked 4/8-lane, small, tiny), the two-class launch, the
             binned launches (split and whole plans), the tile launch (k_span)
             forced and the default dispatch; raw sums with carried parity;
             the dense kernel's shape (it needs a 16-byte-aligned base: an
             unaligned one takes another kernel);
  batchv     checksum and IPv4 multi-batch launches, every class;
  IPv4       COMPUTE / VERIFY / PATCH per segment group, two-class, tile, and
             the tile launch reached through the cached plan (>= 64 Ki
             non-short datagrams, three calls);
  wraps      in place and headers apart, one and two passes, tile;
  routers    in place and headers apart;
  host       the *_host calls from page-locked and pageable buffers at an
             unaligned address (zero-copy and DMA);

and the whole module again under libicsum_debug.so, whose kernels check every
load against the 16-byte blocks that hold the batch's bytes (a read outside
them fails the call): the rebased frame never reads outside the pages the
batch lies in.  Bytes of the allocation outside the batch are checked
untouched.  Bar: bit-exact."""
import numpy as np
import pytest

from conftest import engine_with, force_id
from helpers import pack_contiguous
from test_gpu_parity import _random_datagrams, _t, _u16, _u32

pytestmark = pytest.mark.gpu

BASES = [0, 1, 2, 3, 8, 14]

# one engine per dispatch shape (ICSUM_FORCE test hook), each in the release
# and the bounds-checked build
CSUM_FORCE = [None, {"lps": 16, "unroll": 8, "mode": 3}, {"lps": 64, "unroll": 8, "mode": 3},
              {"lps": 8, "unroll": 8, "mode": 3}, {"lps": 4, "unroll": 2, "mode": 2, "segs": 2},
              {"lps": 1, "unroll": 4, "mode": 4}, {"twoclass": 16}, {"twoclass": 32},
              {"bin": 1, "bin_plan": 1}, {"bin": 1, "bin_plan": 0}, {"bin": 1, "bin_plan": 2},
              {"bin": 1, "bin_plan": 3}, {"tile": 1}, {"tile": 1, "span_segs": 7}]
IPV4_FORCE = [None, {"lps": 16, "unroll": 8, "mode": 3}, {"lps": 4, "unroll": 1, "mode": 2},
              {"lps": 1, "unroll": 4, "mode": 0}, {"twoclass": 16}, {"twoclass": 32}, {"tile": 1},
              {"tile": 1, "span_segs": 1}]
WRAP_FORCE = [None, {"wrap_passes": 1}, {"wrap_passes": 2}, {"tile": 1}, {"tile": 1, "span_segs": 7}]
# fixed-stride batches never take the offsets-only launches (two-class, binned, tile)
CSUM_FIXED_FORCE = [f for f in CSUM_FORCE if not f or not ({"tile", "twoclass", "bin"} & set(f))]
IPV4_FIXED_FORCE = [f for f in IPV4_FORCE if not f or not ({"tile", "twoclass"} & set(f))]


def _ids(p):
    force, debug = p
    return force_id(force or {}) + ("-debug" if debug else "")


def _params(forces):
    return [(f, d) for d in (False, True) for f in forces]


@pytest.fixture(scope="module", params=_params(CSUM_FORCE), ids=_ids)
def csum_eng(request):
    force, debug = request.param
    yield from engine_with(force, debug=debug)


@pytest.fixture(scope="module", params=_params(IPV4_FORCE), ids=_ids)
def ipv4_eng(request):
    force, debug = request.param
    yield from engine_with(force, debug=debug)


@pytest.fixture(scope="module", params=_params(CSUM_FIXED_FORCE), ids=_ids)
def csum_fixed_eng(request):
    force, debug = request.param
    yield from engine_with(force, debug=debug)


@pytest.fixture(scope="module", params=_params(IPV4_FIXED_FORCE), ids=_ids)
def ipv4_fixed_eng(request):
    force, debug = request.param
    yield from engine_with(force, debug=debug)


@pytest.fixture(scope="module", params=_params(WRAP_FORCE), ids=_ids)
def wrap_eng(request):
    force, debug = request.param
    yield from engine_with(force, debug=debug)


@pytest.fixture(scope="module", params=[False, True], ids=["release", "debug"])
def any_eng(request):
    yield from engine_with(None, debug=request.param)


def _place(buf, base):
    """`buf` copied `base` bytes into a fresh device allocation whose other
    bytes are 0xA5; returns (the batch's view, the whole allocation)."""
    import torch

    whole = torch.full((base + buf.size + 64,), 0xA5, dtype=torch.uint8, device="cuda:0")
    whole[base:base + buf.size] = torch.from_numpy(np.ascontiguousarray(buf)).cuda()
    view = whole[base:base + buf.size]
    assert view.data_ptr() % 16 == base % 16  # torch hands out >= 256-byte-aligned blocks
    return view, whole


def _untouched(whole, base, size):
    w = whole.cpu().numpy()
    assert (w[:base] == 0xA5).all() and (w[base + size:] == 0xA5).all()


def _kernel(eng):
    return eng.dispatch_info()["kernel"]


# ---------------------------------------------------------------- checksum --
def _csum_lengths(rng, n):
    """a mix that reaches every per-segment path: ACKs, short, MTU, long, empty"""
    lens = rng.choice([0, 1, 7, 16, 40, 41, 64, 100, 576, 1460, 1500, 3000, 9000], n) + rng.integers(0, 3, n)
    lens[::97] = 0
    return lens


@pytest.mark.parametrize("base", BASES)
def test_checksum_offsets_any_base(csum_eng, orc, base):
    rng = np.random.default_rng(0xBA5E + base)
    n = 3000
    lens = _csum_lengths(rng, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    off += np.uint64(rng.integers(0, 16))  # the first start anywhere in its block too
    buf = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    d, whole = _place(buf, base)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    for call in range(2):  # the second call: from the cached plan where there is one
        out = csum_eng.checksum_batch(d, offsets=_t(off), init=_t(init))
        assert (_u16(out) == orc.checksum_batch(buf, n, offsets=off, init=init)).all(), (base, call, _kernel(csum_eng))
    odd = rng.integers(0, 2, n).astype(np.uint8)
    sums = csum_eng.sum_batch(d, offsets=_t(off), init=_t(init), odd=_t(odd))
    assert (_u32(sums) == orc.sum_batch(buf, n, offsets=off, init=init, odd=odd)).all(), base
    _untouched(whole, base, buf.size)


@pytest.mark.parametrize("base", BASES)
def test_checksum_fixed_stride_any_base(csum_fixed_eng, orc, base):
    eng = csum_fixed_eng
    for stride, seg_len in ((1500, 1500), (1514, 1500), (64, 64), (40, 40), (9000, 9000), (72, 64)):
        rng = np.random.default_rng(stride * 31 + seg_len + base)
        n = 2000
        buf = rng.integers(0, 256, (n - 1) * stride + seg_len, dtype=np.uint8)
        d, whole = _place(buf, base)
        out = eng.checksum_batch(d, n=n, stride=stride, seg_len=seg_len)
        want = orc.checksum_batch(buf, n, stride=stride, seg_len=seg_len)
        assert (_u16(out) == want).all(), (base, stride, seg_len, _kernel(eng))
        _untouched(whole, base, buf.size)


@pytest.mark.parametrize("base", BASES)
def test_dense_shape_any_base(any_eng, orc, base):
    """stride == length == 64 B takes the dense kernel only at a 16-byte-aligned
    base; elsewhere another kernel, with the same results"""
    rng = np.random.default_rng(0xDE + base)
    n = 50_000
    buf = rng.integers(0, 256, n * 64, dtype=np.uint8)
    d, _ = _place(buf, base)
    out = any_eng.checksum_batch(d, n=n, stride=64, seg_len=64)
    assert (_u16(out) == orc.checksum_batch(buf, n, stride=64, seg_len=64)).all(), base
    assert (_kernel(any_eng) == "dense") == (base % 16 == 0), (base, _kernel(any_eng))


@pytest.mark.parametrize("base", [1, 3, 8, 14])
def test_checksum_batchv_any_base(any_eng, orc, base):
    """every checksum multi-batch class (dense-shaped, tiny, small, 16- and
    64-lane line grids, offsets) with each batch at its own unaligned base"""
    import torch

    rng = np.random.default_rng(0xB7 + base)
    batches, wants = [], []
    keep = []
    for k, (stride, L, n) in enumerate(((64, 64, 3000), (40, 40, 5000), (72, 64, 2001), (1500, 1500, 999),
                                        (9000, 9000, 97), (0, 0, 2500))):
        b0 = (base + 3 * k) % 16
        if stride:
            buf = rng.integers(0, 256, (n - 1) * stride + L, dtype=np.uint8)
            d, whole = _place(buf, b0)
            batches.append(dict(data=d, n=n, stride=stride, seg_len=L))
            wants.append(orc.checksum_batch(buf, n, stride=stride, seg_len=L))
        else:
            lens = _csum_lengths(rng, n)
            off = np.zeros(n + 1, dtype=np.uint64)
            off[1:] = np.cumsum(lens)
            buf = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
            d, whole = _place(buf, b0)
            batches.append(dict(data=d, offsets=_t(off)))
            wants.append(orc.checksum_batch(buf, n, offsets=off))
        keep.append(whole)
    outs = any_eng.checksum_batchv(batches)
    torch.cuda.synchronize()
    assert _kernel(any_eng) == "batchv"
    for j, (o, w) in enumerate(zip(outs, wants)):
        assert (_u16(o) == w).all(), (base, j)


# -------------------------------------------------------------------- IPv4 --
def _dgram_arena(rng, n, first):
    segs = _random_datagrams(rng, n)
    return pack_contiguous(segs, first)


def _ipv4_check(eng, orc, buf, off, base, tag):
    n = off.size - 1
    for mode in (0, 1, 2):
        d, whole = _place(buf, base)
        hb = buf.copy()
        want = orc.ipv4_tcp_batch(hb, n, mode, offsets=off)
        ip, tcp, st = eng.ipv4_tcp_batch(d, mode, offsets=_t(off))
        k = _kernel(eng)
        assert (_u16(ip) == want[0]).all(), (tag, base, mode, k)
        assert (_u16(tcp) == want[1]).all(), (tag, base, mode, k)
        assert (st.cpu().numpy() == want[2]).all(), (tag, base, mode, k)
        assert (d.cpu().numpy() == hb).all(), (tag, base, mode, k)  # PATCH: the oracle's bytes
        _untouched(whole, base, buf.size)


@pytest.mark.parametrize("base", BASES)
def test_ipv4_offsets_any_base(ipv4_eng, orc, base):
    """every header shape (options, hlen < 5 and > the datagram, < 20 / < 40
    bytes, bad versions, valid and corrupt checksums) at every start alignment"""
    rng = np.random.default_rng(0x1F4 + base)
    buf, off = _dgram_arena(rng, 2500, int(rng.integers(0, 16)))
    _ipv4_check(ipv4_eng, orc, buf, off, base, "random")


@pytest.mark.parametrize("base", BASES)
def test_ipv4_fixed_stride_any_base(ipv4_fixed_eng, orc, base):
    segs = _random_datagrams(np.random.default_rng(0x1F5 + base), 1000)
    for L in (1500, 1514, 40, 60):
        n = len(segs)
        buf = np.zeros(n * L, dtype=np.uint8)
        for i, sg in enumerate(segs):
            buf[i * L:(i + 1) * L] = np.frombuffer((sg + bytes(L))[:L], dtype=np.uint8)
        for mode in (0, 1, 2):
            d, whole = _place(buf, base)
            hb = buf.copy()
            want = orc.ipv4_tcp_batch(hb, n, mode, stride=L, dgram_len=L)
            ip, tcp, st = ipv4_fixed_eng.ipv4_tcp_batch(d, mode, n=n, stride=L, dgram_len=L)
            assert (_u16(ip) == want[0]).all() and (_u16(tcp) == want[1]).all(), (base, L, mode)
            assert (st.cpu().numpy() == want[2]).all(), (base, L, mode)
            assert (d.cpu().numpy() == hb).all(), (base, L, mode)
            _untouched(whole, base, buf.size)


@pytest.mark.parametrize("base", [1, 2, 3, 8])
def test_ipv4_tile_from_cached_plan_any_base(any_eng, orc, base):
    """The default dispatch runs an offsets batch of >= 64 Ki non-short
    datagrams (40..1040 bytes, the transmit mix) through the tile launch from
    its cached plan: k_span's header read (the IHL that places the TCP part)
    at an unaligned base, three calls per mode, every result the oracle's."""
    rng = np.random.default_rng(0x7B + base)
    n = 70_000
    lens = 40 + rng.integers(0, 1001, n)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum(lens)
    buf = rng.integers(0, 256, int(off[-1]), dtype=np.uint8)
    s = off[:-1].astype(np.int64)
    hl = rng.choice([5, 5, 5, 6, 7, 15, 4], n)  # options, and header lengths past short datagrams
    buf[s] = (0x40 | hl).astype(np.uint8)
    buf[s + 2], buf[s + 3] = (lens >> 8).astype(np.uint8), (lens & 255).astype(np.uint8)
    buf[s + 6], buf[s + 8], buf[s + 9] = 0x40, 64, 6
    orc.ipv4_tcp_batch(buf, n, 2, offsets=off)  # valid checksums
    buf[s[::11] + 30] ^= 0x20  # some corrupt TCP bytes
    d, whole = _place(buf, base)
    do = _t(off)
    hb = buf.copy()
    kinds = []
    for mode in (1, 0, 2):
        for call in range(3):
            want = orc.ipv4_tcp_batch(hb, n, mode, offsets=off)
            ip, tcp, st = any_eng.ipv4_tcp_batch(d, mode, offsets=do)
            kinds.append(_kernel(any_eng))
            assert (_u16(ip) == want[0]).all() and (_u16(tcp) == want[1]).all(), (base, mode, call, kinds[-1])
            assert (st.cpu().numpy() == want[2]).all(), (base, mode, call)
            assert (d.cpu().numpy() == hb).all(), (base, mode, call)
    assert kinds[2:] == ["tile"] * 7, kinds
    _untouched(whole, base, buf.size)


@pytest.mark.parametrize("base", [1, 3, 8, 14])
def test_ipv4_batchv_any_base(any_eng, orc, base):
    import torch

    rng = np.random.default_rng(0x1B7 + base)
    hosts = []
    for k, (L, n) in enumerate(((1500, 800), (40, 3000), (9000, 60), (0, 1500))):
        b0 = (base + 5 * k) % 16
        if L:
            segs = _random_datagrams(rng, n)
            buf = np.zeros(n * L, dtype=np.uint8)
            for i, sg in enumerate(segs):
                buf[i * L:(i + 1) * L] = np.frombuffer((sg + bytes(L))[:L], dtype=np.uint8)
            hosts.append(dict(buf=buf, n=n, stride=L, dgram_len=L, offsets=None, base=b0))
        else:
            buf, off = _dgram_arena(rng, n, 0)
            hosts.append(dict(buf=buf, n=n, stride=0, dgram_len=0, offsets=off, base=b0))
    placed = [_place(h["buf"], h["base"]) for h in hosts]
    for mode in (0, 1, 2):
        wants = []
        for h in hosts:
            if h["offsets"] is None:
                wants.append(orc.ipv4_tcp_batch(h["buf"], h["n"], mode, stride=h["stride"], dgram_len=h["dgram_len"]))
            else:
                wants.append(orc.ipv4_tcp_batch(h["buf"], h["n"], mode, offsets=h["offsets"]))
        batches = [dict(dgrams=p[0], n=h["n"], stride=h["stride"], dgram_len=h["dgram_len"],
                        offsets=None if h["offsets"] is None else _t(h["offsets"])) for p, h in zip(placed, hosts)]
        outs = any_eng.ipv4_tcp_batchv(batches, mode)
        torch.cuda.synchronize()
        for j, ((ip, tcp, st), w, p, h) in enumerate(zip(outs, wants, placed, hosts)):
            assert (_u16(ip) == w[0]).all() and (_u16(tcp) == w[1]).all(), (base, mode, j)
            assert (st.cpu().numpy() == w[2]).all(), (base, mode, j)
            assert (p[0].cpu().numpy() == h["buf"]).all(), (base, mode, j)


# ------------------------------------------------------------------- wraps --
@pytest.mark.parametrize("base", BASES)
def test_wrap_in_place_any_base(wrap_eng, orc, base):
    import torch

    from test_gpu_wrap import _oracle_wire, _random_batch

    rng = np.random.default_rng(0x3A + base)
    segs, m = _random_batch(rng, 1500)
    segs += [b"\x5a" * 39, b""]  # shorter than 40: untouched
    m = np.concatenate([m, m[:2]])
    want = _oracle_wire(orc, segs[:-2], m[:-2]) + segs[-2:]
    buf, off = pack_contiguous(segs, int(rng.integers(0, 16)))
    buf = buf[:int(off[-1])].copy()
    d, whole = _place(buf, base)
    wrap_eng.tcp_wrap_batch(d, torch.from_numpy(m.view(np.uint8).copy()).cuda(), n=len(segs), offsets=_t(off))
    got = d.cpu().numpy()
    for i, w in enumerate(want):
        assert got[off[i]:off[i + 1]].tobytes() == w, (base, i, _kernel(wrap_eng))
    _untouched(whole, base, buf.size)
    if wrap_eng.forced.get("tile"):
        return
    # fixed stride: every datagram start at the base's alignment (+ k * 1040)
    L, n = 1040, 600
    _, m2 = _random_batch(rng, n, fixed=L - 40)
    body = rng.integers(0, 256, n * L, dtype=np.uint8)
    d, whole = _place(body, base)
    wrap_eng.tcp_wrap_batch(d, torch.from_numpy(m2.view(np.uint8).copy()).cuda(), n=n, stride=L, dgram_len=L)
    got = d.cpu().numpy()
    for i in range(0, n, 7):
        w = _oracle_wire(orc, [b"\0" * 40 + body[i * L + 40:(i + 1) * L].tobytes()], m2[i:i + 1])[0]
        assert got[i * L:(i + 1) * L].tobytes() == w, (base, i)
    _untouched(whole, base, body.size)


@pytest.mark.parametrize("base", BASES)
def test_wrap_headers_apart_any_base(wrap_eng, orc, base):
    import torch

    from test_gpu_wrap import _oracle_wire, _random_batch

    rng = np.random.default_rng(0x3B + base)
    segs, m = _random_batch(rng, 1500)
    want = _oracle_wire(orc, segs, m)
    buf, off = pack_contiguous([s[40:] for s in segs], int(rng.integers(0, 16)))
    buf = buf[:int(off[-1])].copy()
    d, whole = _place(buf, base)
    hd = torch.zeros(len(segs) * 40, dtype=torch.uint8, device="cuda")
    wrap_eng.tcp_wrap_headers(d, torch.from_numpy(m.view(np.uint8).copy()).cuda(), hd, n=len(segs), offsets=_t(off))
    h = hd.cpu().numpy()
    for i, w in enumerate(want):
        assert h[40 * i:40 * i + 40].tobytes() == w[:40], (base, i, _kernel(wrap_eng))
    assert (d.cpu().numpy() == buf).all()  # payloads only read
    _untouched(whole, base, buf.size)


# ----------------------------------------------------------------- routers --
def _router_arena(rng, orc, n):
    segs = _random_datagrams(rng, n)
    for i in range(0, len(segs), 2):  # valid headers with every ttl: forwards and drops
        if len(segs[i]) >= 20:
            b = bytearray(segs[i])
            b[0] = 0x45
            b[6] |= 0x80 if i % 6 == 0 else 0  # reserved flag bit: dropped on the way out
            b[8] = i % 256
            _, _, _, b = orc.ipv4_tcp(bytes(b), 2)
            segs[i] = b
    return segs


@pytest.mark.parametrize("base", BASES)
def test_router_both_forms_any_base(any_eng, orc, base):
    import torch

    from test_gpu_router_hdrs import _want_hdrs

    rng = np.random.default_rng(0x40 + base)
    segs = _router_arena(rng, orc, 2000)
    buf, off = pack_contiguous(segs, int(rng.integers(0, 16)))
    buf = buf[:int(off[-1])].copy()
    n = len(segs)
    st_want, hd_want = _want_hdrs(orc, buf, off)
    hb = buf.copy()
    for i in range(n):
        a, b = int(off[i]), int(off[i + 1])
        _, out = orc.router_ttl(hb[a:b].tobytes())
        hb[a:b] = np.frombuffer(out, dtype=np.uint8)
    # headers apart: the datagrams only read
    d, whole = _place(buf, base)
    hd = torch.full((n * 20,), 0xA5, dtype=torch.uint8, device="cuda:0")
    hd, st = any_eng.router_ttl_headers(d, offsets=_t(off), hdrs=hd)
    assert st.cpu().numpy().tolist() == st_want and (hd.cpu().numpy() == hd_want).all(), base
    assert (d.cpu().numpy() == buf).all()
    # in place
    st = any_eng.router_ttl_batch(d, offsets=_t(off)).cpu().numpy()
    assert st.tolist() == st_want, base
    assert (d.cpu().numpy() == hb).all(), base
    _untouched(whole, base, buf.size)
    # fixed stride 1514: header starts at every alignment the base gives
    L = 1514
    fb = np.zeros(300 * L, dtype=np.uint8)
    for i, sg in enumerate(_router_arena(rng, orc, 300)):
        fb[i * L:(i + 1) * L] = np.frombuffer((bytes(sg) + bytes(L))[:L], dtype=np.uint8)
    d, whole = _place(fb, base)
    st = any_eng.router_ttl_batch(d, n=300, stride=L, dgram_len=L).cpu().numpy()
    want = []
    fh = fb.copy()
    for i in range(300):
        f, out = orc.router_ttl(fh[i * L:(i + 1) * L].tobytes())
        fh[i * L:(i + 1) * L] = np.frombuffer(out, dtype=np.uint8)
        want.append(f)
    assert st.tolist() == want and (d.cpu().numpy() == fh).all(), base
    _untouched(whole, base, fb.size)


# -------------------------------------------------------------------- host --
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("base", [1, 3, 14])
@pytest.mark.parametrize("n", [8, 20_000])  # one zero-copy launch / DMA'd chunks
def test_host_calls_any_base(any_eng, orc, base, pinned, n):
    """*_host calls on a buffer that starts `base` bytes into a host
    allocation: page-locked batches of <= 2 MiB are read in place by the
    kernel (zero-copy), larger ones DMA'd from that address"""
    import torch

    rng = np.random.default_rng(0x405 + base + n)
    L = 1514
    segs = _random_datagrams(rng, n)
    flat = np.zeros(n * L, dtype=np.uint8)
    for i, sg in enumerate(segs):
        flat[i * L:(i + 1) * L] = np.frombuffer((sg + bytes(L))[:L], dtype=np.uint8)
    alloc = torch.empty(flat.size + base + 64, dtype=torch.uint8, pin_memory=pinned).numpy()
    alloc[:] = 0xA5
    h = alloc[base:base + flat.size]
    for mode in (1, 2):
        h[:] = flat
        hb = flat.copy()
        want = orc.ipv4_tcp_batch(hb, n, mode, stride=L, dgram_len=L)
        ip, tcp, st = any_eng.ipv4_tcp_batch_host(h, n, mode, stride=L, dgram_len=L)
        assert (ip == want[0]).all() and (tcp == want[1]).all() and (st == want[2]).all(), (base, mode)
        assert (h == hb).all(), (base, mode)
    out = any_eng.checksum_batch_host(h, n, stride=L, seg_len=L - 3)
    assert (out == orc.checksum_batch(h, n, stride=L, seg_len=L - 3)).all(), base
    assert (alloc[:base] == 0xA5).all() and (alloc[base + flat.size:] == 0xA5).all()
