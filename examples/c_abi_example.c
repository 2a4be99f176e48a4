/* c_abi_example.c — the C-ABI (include/icsum.h) from plain C11, as
 * INTEGRATION.md §3 shows it: a complete program rather than a fragment.
 * tests/test_c_example.py compiles it with -std=c11 -pedantic -Werror (no GPU
 * needed); tests/test_gpu_c_example.py runs it and checks every printed value
 * against the oracle.  Built in-tree by `make -C examples` (build() does it).
 *
 * Output, one result per line:
 *   checksum <i> <u16>                 ics_checksum_batch, fixed stride + inits
 *   batchv <i> <u16>                   the same bytes as two batches in one ics_checksum_batchv
 *   patch <i> <ip u16> <tcp u16>       ics_ipv4_tcp_batch_host, PATCH, packed offsets
 *   verify <i> <status>                then VERIFY of the patched bytes
 *   wrap <i> <hex of the datagram>     ics_tcp_wrap_batch_host: both headers + both checksums */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "icsum.h"

#define CHECK(call)                                                           \
  do {                                                                        \
    int rc_ = (call);                                                         \
    if (rc_ != ICS_OK) {                                                      \
      fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, ics_last_error()); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

enum { N_SEG = 1000, SEG = 100, N_DG = 64, N_WRAP = 8 };

/* the byte / init patterns the test restates */
static uint8_t byte_at(uint64_t i) { return (uint8_t)((i * 2654435761u) >> 13); }
static uint32_t init_at(uint64_t i) { return (uint32_t)(i * 40503u); }
static uint64_t dgram_len(uint64_t i) { return 40 + (i * 7) % 60; }

static int checksums(ics_ctx* ctx) {
  static uint8_t bytes[N_SEG * SEG];
  static uint32_t init[N_SEG];
  static uint16_t out[N_SEG], outv[N_SEG];
  for (uint64_t i = 0; i < sizeof bytes; ++i) bytes[i] = byte_at(i);
  for (uint64_t i = 0; i < N_SEG; ++i) init[i] = init_at(i);
  void *d_bytes = NULL, *d_init = NULL, *d_out = NULL, *d_outv = NULL;
  CHECK(ics_malloc(ctx, &d_bytes, sizeof bytes));
  CHECK(ics_malloc(ctx, &d_init, sizeof init));
  CHECK(ics_malloc(ctx, &d_out, sizeof out));
  CHECK(ics_malloc(ctx, &d_outv, sizeof outv));
  CHECK(ics_memcpy_htod(ctx, d_bytes, bytes, sizeof bytes, NULL));
  CHECK(ics_memcpy_htod(ctx, d_init, init, sizeof init, NULL));
  /* one batch: N_SEG segments of SEG bytes, SEG apart, pseudo-header inits */
  CHECK(ics_checksum_batch(ctx, d_bytes, NULL, SEG, SEG, (const uint32_t*)d_init, (uint16_t*)d_out, N_SEG, NULL));
  /* the same segments as two batches handed over together: one launch */
  const uint64_t half = N_SEG / 2;
  ics_seg_batch b[2] = {
      {d_bytes, NULL, SEG, SEG, half, (const uint32_t*)d_init, (uint16_t*)d_outv},
      {(const uint8_t*)d_bytes + half * SEG, NULL, SEG, SEG, N_SEG - half, (const uint32_t*)d_init + half,
       (uint16_t*)d_outv + half},
  };
  CHECK(ics_checksum_batchv(ctx, b, 2, NULL));
  CHECK(ics_memcpy_dtoh(ctx, out, d_out, sizeof out, NULL));
  CHECK(ics_memcpy_dtoh(ctx, outv, d_outv, sizeof outv, NULL));
  CHECK(ics_stream_synchronize(ctx, NULL));
  for (int i = 0; i < N_SEG; ++i) printf("checksum %d %u\n", i, (unsigned)out[i]);
  for (int i = 0; i < N_SEG; ++i) printf("batchv %d %u\n", i, (unsigned)outv[i]);
  CHECK(ics_free(ctx, d_bytes));
  CHECK(ics_free(ctx, d_init));
  CHECK(ics_free(ctx, d_out));
  CHECK(ics_free(ctx, d_outv));
  return 0;
}

static int datagrams(ics_ctx* ctx) {
  /* N_DG raw IPv4/TCP datagrams back to back (packed offsets, lengths 40-99),
   * in host memory: IPv4 ver 4 / hlen 5 / total length / id i / proto 6, TCP
   * data offset 5, the other bytes from the pattern */
  uint64_t off[N_DG + 1];
  off[0] = 0;
  for (int i = 0; i < N_DG; ++i) off[i + 1] = off[i] + dgram_len((uint64_t)i);
  uint8_t* wire = malloc(off[N_DG]);
  if (!wire) return 1;
  for (uint64_t j = 0; j < off[N_DG]; ++j) wire[j] = byte_at(j + 7);
  for (int i = 0; i < N_DG; ++i) {
    uint8_t* d = wire + off[i];
    const uint64_t len = dgram_len((uint64_t)i);
    d[0] = 0x45;
    d[2] = (uint8_t)(len >> 8);
    d[3] = (uint8_t)len;
    d[4] = 0;
    d[5] = (uint8_t)i;
    d[6] = 0x40;
    d[7] = 0;
    d[9] = 6;
    d[32] = 0x50;
  }
  uint16_t ip[N_DG], tcp[N_DG];
  uint8_t st[N_DG];
  /* PATCH: both checksum fields written into the caller's bytes */
  CHECK(ics_ipv4_tcp_batch_host(ctx, wire, off, 0, 0, N_DG, ICS_MODE_PATCH, ip, tcp, st));
  for (int i = 0; i < N_DG; ++i) printf("patch %d %u %u\n", i, (unsigned)ip[i], (unsigned)tcp[i]);
  /* VERIFY of the patched bytes: every datagram is accepted */
  CHECK(ics_ipv4_tcp_batch_host(ctx, wire, off, 0, 0, N_DG, ICS_MODE_VERIFY, ip, tcp, st));
  for (int i = 0; i < N_DG; ++i) printf("verify %d %u\n", i, (unsigned)st[i]);
  free(wire);
  return 0;
}

static int wrap(ics_ctx* ctx) {
  /* wrap_tcp_in_ip for N_WRAP messages: datagram i = 40 bytes of header room
   * + a payload of 3 i bytes; the engine writes both headers and checksums */
  uint64_t off[N_WRAP + 1];
  off[0] = 0;
  for (int i = 0; i < N_WRAP; ++i) off[i + 1] = off[i] + 40 + 3 * (uint64_t)i;
  uint8_t arena[N_WRAP * 40 + 3 * N_WRAP * N_WRAP];
  memset(arena, 0, sizeof arena);
  for (int i = 0; i < N_WRAP; ++i)
    for (uint64_t j = 0; j < 3 * (uint64_t)i; ++j) arena[off[i] + 40 + j] = byte_at(1000 + 64 * (uint64_t)i + j);
  ics_tcp_msg msgs[N_WRAP];
  memset(msgs, 0, sizeof msgs);
  for (int i = 0; i < N_WRAP; ++i) {
    msgs[i].src = 0x0A000001u + (uint32_t)i;
    msgs[i].dst = 0x0A0000FEu;
    msgs[i].seqno = 1000u * (uint32_t)i + 17u;
    msgs[i].ackno = (i % 2) ? 5000u + (uint32_t)i : 0u;
    msgs[i].src_port = (uint16_t)(40000 + i);
    msgs[i].dst_port = 80;
    msgs[i].window = (uint16_t)(4096 * i + 1);
    msgs[i].flags = (uint8_t)((i % 2 ? ICS_TCP_ACK : 0u) | (i == 0 ? ICS_TCP_SYN : 0u) | (i == 7 ? ICS_TCP_FIN : 0u));
    msgs[i].ttl = 128;
    msgs[i].id = 0;
  }
  CHECK(ics_tcp_wrap_batch_host(ctx, arena, off, 0, 0, N_WRAP, msgs));
  for (int i = 0; i < N_WRAP; ++i) {
    printf("wrap %d ", i);
    for (uint64_t j = off[i]; j < off[i + 1]; ++j) printf("%02x", arena[j]);
    printf("\n");
  }
  return 0;
}

int main(void) {
  ics_ctx* ctx = NULL;
  CHECK(ics_create(0, &ctx));
  int rc = checksums(ctx);
  if (!rc) rc = datagrams(ctx);
  if (!rc) rc = wrap(ctx);
  CHECK(ics_destroy(ctx));
  return rc;
}
