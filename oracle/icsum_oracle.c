/*
 * icsum_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker, CPU baseline "port").
 *
 * A plain-C restatement of the reference's checksum path, written from the
 * semantics (not the text) of:
 *   util/tools/checksum.h:9-60            InternetChecksum
 *   util/ipv4_header/ipv4_header.cpp:9-123 IPv4Header parse/serialize/pseudo/compute
 *   util/tcp_segment/tcp_segment.cpp:9-118 TCPSegment parse (verify) / compute
 *   src/router/router.cpp:43-50            ttl-- + header recompute
 * Deliberately byte-serial like the reference (checksum.h:22-27) so that its
 * speed is representative of the reference CPU path.
 * Pinned against the real reference via tests/golden/ (oracle/make_golden.py).
 */
#include "icsum_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- a1-a4 -- */

/* checksum.h:17 — explicit InternetChecksum(uint32_t sum = 0) */
void orc_init(orc_cksum* c, uint32_t init) {
    c->sum = init;
    c->parity = 0;
}

/* checksum.h:20-28 — each byte is the high half of a 16-bit word when the
 * running parity is even, the low half when odd; uint32 wrapping add. */
void orc_add(orc_cksum* c, const uint8_t* data, size_t n) {
    uint32_t s = c->sum;
    int odd = c->parity;
    for (size_t i = 0; i < n; ++i) {
        const uint32_t b = data[i];
        s += odd ? b : (b << 8);
        odd ^= 1;
    }
    c->sum = s;
    c->parity = odd;
}

/* checksum.h:31-41 — end-around-carry fold until it fits 16 bits, then ~. */
uint16_t orc_fold(uint32_t sum) {
    uint32_t r = sum;
    while (r > 0xffffu) r = (r >> 16) + (r & 0xffffu);
    return (uint16_t)~r;
}

uint16_t orc_value(const orc_cksum* c) { return orc_fold(c->sum); }

static void seg_bounds(const uint64_t* offsets, uint64_t stride, uint64_t seg_len, uint64_t i,
                       uint64_t* b, uint64_t* e) {
    if (offsets) {
        *b = offsets[i];
        *e = offsets[i + 1];
    } else {
        *b = i * stride;
        *e = *b + seg_len;
    }
}

void orc_checksum_batch(const uint8_t* bytes, const uint64_t* offsets, uint64_t stride,
                        uint64_t seg_len, const uint32_t* init, uint16_t* out, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t b, e;
        seg_bounds(offsets, stride, seg_len, i, &b, &e);
        orc_cksum c;
        orc_init(&c, init ? init[i] : 0u);
        orc_add(&c, bytes + b, (size_t)(e - b));
        out[i] = orc_value(&c);
    }
}

void orc_sum_batch(const uint8_t* bytes, const uint64_t* offsets, uint64_t stride,
                   uint64_t seg_len, const uint32_t* init, const uint8_t* odd, uint32_t* sums,
                   uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t b, e;
        seg_bounds(offsets, stride, seg_len, i, &b, &e);
        orc_cksum c;
        orc_init(&c, init ? init[i] : 0u);
        c.parity = odd ? (odd[i] & 1) : 0;
        orc_add(&c, bytes + b, (size_t)(e - b));
        sums[i] = c.sum;
    }
}

typedef struct {
    const uint8_t* bytes;
    const uint64_t* offsets;
    uint64_t stride, seg_len;
    const uint32_t* init;
    uint16_t* out;
    uint64_t lo, hi;
} mt_job;

static void* mt_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        uint64_t b, e;
        seg_bounds(j->offsets, j->stride, j->seg_len, i, &b, &e);
        orc_cksum c;
        orc_init(&c, j->init ? j->init[i] : 0u);
        orc_add(&c, j->bytes + b, (size_t)(e - b));
        j->out[i] = orc_value(&c);
    }
    return NULL;
}

int orc_checksum_batch_mt(const uint8_t* bytes, const uint64_t* offsets, uint64_t stride,
                          uint64_t seg_len, const uint32_t* init, uint16_t* out, uint64_t n,
                          int threads) {
    if (threads < 1) threads = 1;
    if (threads == 1 || n < (uint64_t)threads) {
        orc_checksum_batch(bytes, offsets, stride, seg_len, init, out, n);
        return 0;
    }
    pthread_t* tid = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    mt_job* jobs = (mt_job*)calloc((size_t)threads, sizeof(mt_job));
    char* started = (char*)calloc((size_t)threads, 1);
    if (!tid || !jobs || !started) {
        free(tid);
        free(jobs);
        free(started);
        return -1;
    }
    for (int t = 0; t < threads; ++t) {
        mt_job* j = &jobs[t];
        j->bytes = bytes;
        j->offsets = offsets;
        j->stride = stride;
        j->seg_len = seg_len;
        j->init = init;
        j->out = out;
        j->lo = n * (uint64_t)t / (uint64_t)threads;
        j->hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        if (pthread_create(&tid[t], NULL, mt_worker, j) != 0) {
            mt_worker(j); /* run inline if a thread cannot be started */
            started[t] = 0;
        } else {
            started[t] = 1;
        }
    }
    for (int t = 0; t < threads; ++t)
        if (started[t]) pthread_join(tid[t], NULL);
    free(tid);
    free(jobs);
    free(started);
    return 0;
}

/* ------------------------------------------------------ IPv4 + TCP ------ */

#define ST_IPV4_OK 0x01u
#define ST_TCP_CKSUM_OK 0x02u
#define ST_TCP_HDR_OK 0x04u
#define ST_PROTO_TCP 0x08u

static uint32_t rd16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }
static uint32_t rd32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static void wr16(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
static void wr32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

typedef struct {
    uint32_t ver, hlen, tos, len, id, df, mf, offset, ttl, proto, cksum, src, dst;
} ipv4_fields;

/* ipv4_header.cpp:9-30 — field extraction from the first 20 wire bytes. */
static void ipv4_parse_fields(const uint8_t* d, ipv4_fields* h) {
    h->ver = d[0] >> 4;
    h->hlen = d[0] & 0x0fu;
    h->tos = d[1];
    h->len = rd16(d + 2);
    h->id = rd16(d + 4);
    const uint32_t fo = rd16(d + 6);
    h->df = (fo & 0x4000u) != 0;
    h->mf = (fo & 0x2000u) != 0;
    h->offset = fo & 0x1fffu;
    h->ttl = d[8];
    h->proto = d[9];
    h->cksum = rd16(d + 10);
    h->src = rd32(d + 12);
    h->dst = rd32(d + 16);
}

/* ipv4_header.cpp:62-86 + :113-123 — serialize the fields (cksum 0, the
 * reserved flag bit is not representable, options never emitted) and sum. */
static uint16_t ipv4_compute(const ipv4_fields* h) {
    uint8_t s[20];
    s[0] = (uint8_t)((h->ver << 4) | (h->hlen & 0x0fu));
    s[1] = (uint8_t)h->tos;
    wr16(s + 2, h->len);
    wr16(s + 4, h->id);
    wr16(s + 6, (h->df ? 0x4000u : 0u) | (h->mf ? 0x2000u : 0u) | (h->offset & 0x1fffu));
    s[8] = (uint8_t)h->ttl;
    s[9] = (uint8_t)h->proto;
    s[10] = 0;
    s[11] = 0;
    wr32(s + 12, h->src);
    wr32(s + 16, h->dst);
    orc_cksum c;
    orc_init(&c, 0);
    orc_add(&c, s, 20);
    return orc_value(&c);
}

/* ipv4_header.cpp:89-110 — payload_length() wraps mod 2^16; unfolded sum. */
static uint32_t ipv4_pseudo(const ipv4_fields* h) {
    const uint16_t plen = (uint16_t)(h->len - 4u * h->hlen);
    uint32_t p = (h->src >> 16) + (h->src & 0xffffu);
    p += (h->dst >> 16) + (h->dst & 0xffffu);
    p += h->proto;
    p += plen;
    return p;
}

void orc_ipv4_tcp(uint8_t* d, uint64_t L, int mode, uint16_t* ip_ck, uint16_t* tcp_ck,
                  uint8_t* status) {
    if (L < 20) {
        *ip_ck = 0;
        *tcp_ck = 0;
        *status = 0;
        return;
    }
    ipv4_fields h;
    ipv4_parse_fields(d, &h);
    const uint16_t ipc = ipv4_compute(&h);
    const int hdr_ok = (h.ver == 4) && (h.hlen >= 5); /* ipv4_header.cpp:32-41 */
    const uint32_t pseudo = ipv4_pseudo(&h);
    uint64_t off = 4u * (uint64_t)h.hlen; /* options skipped, ipv4_header.cpp:50 */
    if (off < 20) off = 20;
    if (off > L) off = L;
    const uint64_t rem = L - off;
    const uint8_t* t = d + off;
    uint8_t st = 0;
    if (h.proto == 6) st |= ST_PROTO_TCP; /* tcp_over_ip.cpp:26-29 */
    if (rem >= 20 && (t[12] >> 4) >= 5) st |= ST_TCP_HDR_OK; /* tcp_segment.cpp:25-65 */
    orc_cksum c;
    orc_init(&c, pseudo);
    uint16_t tv;
    if (mode == 1) {
        /* tcp_segment.cpp:11-18 — all remaining bytes, value()==0 */
        orc_add(&c, t, (size_t)rem);
        tv = orc_value(&c);
        if (hdr_ok && ipc == h.cksum) st |= ST_IPV4_OK; /* ipv4_header.cpp:53-58 */
        if (tv == 0) st |= ST_TCP_CKSUM_OK;
    } else {
        /* tcp_segment.cpp:109-118 — udinfo.cksum = 0 while summing */
        static const uint8_t zero2[2] = {0, 0};
        const uint64_t a = rem < 16 ? rem : 16;
        orc_add(&c, t, (size_t)a);
        if (rem > 16) orc_add(&c, zero2, rem > 17 ? 2 : 1);
        if (rem > 18) orc_add(&c, t + 18, (size_t)(rem - 18));
        tv = orc_value(&c);
        if (hdr_ok) st |= ST_IPV4_OK;
        if (rem >= 18) st |= ST_TCP_CKSUM_OK;
        if (mode == 2) {
            wr16(d + 10, ipc);
            if (rem >= 18) wr16(d + off + 16, tv);
        }
    }
    *ip_ck = ipc;
    *tcp_ck = tv;
    *status = st;
}

void orc_ipv4_tcp_batch(uint8_t* dgrams, const uint64_t* offsets, uint64_t stride,
                        uint64_t dgram_len, uint64_t n, int mode, uint16_t* ip_ck,
                        uint16_t* tcp_ck, uint8_t* status) {
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t b, e;
        seg_bounds(offsets, stride, dgram_len, i, &b, &e);
        uint16_t a, t;
        uint8_t s;
        orc_ipv4_tcp(dgrams + b, e - b, mode, &a, &t, &s);
        if (ip_ck) ip_ck[i] = a;
        if (tcp_ck) tcp_ck[i] = t;
        if (status) status[i] = s;
    }
}

/* network_interface.cpp:51 (parse = verify) then router.cpp:43-50. */
void orc_router_ttl(uint8_t* d, uint64_t L, uint8_t* status) {
    *status = 0;
    if (L < 20) return;
    ipv4_fields h;
    ipv4_parse_fields(d, &h);
    if (h.ver != 4 || h.hlen < 5) return;
    if (ipv4_compute(&h) != h.cksum) return;
    if (h.ttl <= 1) return;
    h.ttl -= 1;
    const uint16_t c = ipv4_compute(&h);
    /* the forwarded header is the re-serialized one: ttl, checksum, and the
     * flags word without the reserved bit (ipv4_header.cpp:78). */
    d[6] &= 0x7fu;
    d[8] = (uint8_t)h.ttl;
    wr16(d + 10, c);
    *status = 1;
}

/* ---------------------------------------------------- workload spec ---- */

#define SPEC_GOLDEN 0x9E3779B97F4A7C15ull

uint64_t orc_sm64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint64_t orc_word(uint64_t seed, uint64_t c) { return orc_sm64(seed + (c + 1) * SPEC_GOLDEN); }

void orc_fill_bytes(uint64_t seed, uint64_t pos0, uint64_t n, uint8_t* out) {
    uint64_t j = 0;
    /* byte p of the stream is byte (p & 7) of word p >> 3, little-endian */
    while (j < n && ((pos0 + j) & 7)) {
        const uint64_t p = pos0 + j;
        out[j++] = (uint8_t)(orc_word(seed, p >> 3) >> (8 * (p & 7)));
    }
    while (j + 8 <= n) {
        const uint64_t w = orc_word(seed, (pos0 + j) >> 3);
        for (int k = 0; k < 8; ++k) out[j + k] = (uint8_t)(w >> (8 * k));
        j += 8;
    }
    while (j < n) {
        const uint64_t p = pos0 + j;
        out[j++] = (uint8_t)(orc_word(seed, p >> 3) >> (8 * (p & 7)));
    }
}

static uint64_t spec_meta(uint64_t seed, uint64_t i) {
    return orc_word(seed ^ 0xA5A5A5A5A5A5A5A5ull, i);
}

static void spec_addrs(uint64_t seed, uint64_t i, uint32_t* src, uint32_t* dst) {
    const uint64_t m = spec_meta(seed, i);
    *src = 0x0A000000u | (uint32_t)(m & 0xFFFFFFu);
    *dst = 0x0A000000u | (uint32_t)((m >> 24) & 0xFFFFFFu);
}

uint32_t orc_pseudo_init(uint64_t seed, uint64_t i, uint64_t len) {
    uint32_t s, d;
    spec_addrs(seed, i, &s, &d);
    return (s >> 16) + (s & 0xffffu) + (d >> 16) + (d & 0xffffu) + 6u + (uint32_t)(len & 0xffffu);
}

uint64_t orc_mixed_len(uint64_t seed, uint64_t i) {
    const uint64_t m = orc_word(seed ^ 0x3C3C3C3C3C3C3C3Cull, i);
    const unsigned e = 6u + (unsigned)(m % 10u);
    return (1ull << e) + ((m >> 8) & ((1ull << e) - 1));
}

void orc_ipv4_tcp_headers(uint64_t seed, uint64_t i, uint64_t dgram_len, uint8_t* d) {
    uint32_t s, t;
    spec_addrs(seed, i, &s, &t);
    d[0] = 0x45;
    d[1] = 0;
    wr16(d + 2, (uint32_t)(dgram_len & 0xffffu));
    wr16(d + 4, (uint32_t)(i & 0xffffu));
    d[6] = 0x40;
    d[7] = 0;
    d[8] = 64;
    d[9] = 6;
    wr32(d + 12, s);
    wr32(d + 16, t);
    if (dgram_len >= 40) {
        d[32] = 0x50;
        d[33] = 0x10;
        d[38] = 0;
        d[39] = 0;
    }
}
