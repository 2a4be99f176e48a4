/*
 * icsum_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Internet-checksum path, used as the parity
 * checker for the HIP engine.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product (libicsum.so and the
 * host C++ types) never links or calls it.
 *
 * Pinning: this restatement is checked against golden vectors produced by the
 * real reference compiled from /root/reference (oracle/ref/, fixtures in
 * tests/golden/, generator oracle/make_golden.py) — see DESIGN.md §Oracle.
 */
#ifndef ICSUM_ORACLE_H
#define ICSUM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* util/tools/checksum.h:9-60 — InternetChecksum state */
typedef struct {
    uint32_t sum;   /* sum_    (checksum.h:12) */
    int parity;     /* parity_ (checksum.h:13) */
} orc_cksum;

void orc_init(orc_cksum* c, uint32_t init);                /* checksum.h:17 */
void orc_add(orc_cksum* c, const uint8_t* data, size_t n); /* checksum.h:20-28 */
uint16_t orc_value(const orc_cksum* c);                    /* checksum.h:31-41 */
uint16_t orc_fold(uint32_t sum);                           /* value() of a raw sum */

/* Batch forms (segment addressing as in include/icsum.h). */
void orc_checksum_batch(const uint8_t* bytes, const uint64_t* offsets, uint64_t stride,
                        uint64_t seg_len, const uint32_t* init, uint16_t* out, uint64_t n);
void orc_sum_batch(const uint8_t* bytes, const uint64_t* offsets, uint64_t stride,
                   uint64_t seg_len, const uint32_t* init, const uint8_t* odd, uint32_t* sums,
                   uint64_t n);
/* Same as orc_checksum_batch split over `threads` pthreads (contiguous index
 * ranges).  Returns 0 on success. */
int orc_checksum_batch_mt(const uint8_t* bytes, const uint64_t* offsets, uint64_t stride,
                          uint64_t seg_len, const uint32_t* init, uint16_t* out, uint64_t n,
                          int threads);

/* IPv4 header + TCP (ipv4_header.cpp:9-123, tcp_segment.cpp:9-118):
 * one raw datagram, modes/status bits as ICS_MODE_* / ICS_ST_* in icsum.h.
 * In PATCH mode (2) the datagram bytes are modified in place. */
void orc_ipv4_tcp(uint8_t* dgram, uint64_t len, int mode, uint16_t* ip_ck, uint16_t* tcp_ck,
                  uint8_t* status);
void orc_ipv4_tcp_batch(uint8_t* dgrams, const uint64_t* offsets, uint64_t stride,
                        uint64_t dgram_len, uint64_t n, int mode, uint16_t* ip_ck,
                        uint16_t* tcp_ck, uint8_t* status);
/* src/router/router.cpp:43-50 on one raw datagram (status 1 forwarded, 0 not). */
void orc_router_ttl(uint8_t* dgram, uint64_t len, uint8_t* status);

/* ---- workload spec (DESIGN.md §Workload spec) ---------------------------- */
uint64_t orc_sm64(uint64_t z);
uint64_t orc_word(uint64_t seed, uint64_t c);
void orc_fill_bytes(uint64_t seed, uint64_t pos0, uint64_t n, uint8_t* out);
uint32_t orc_pseudo_init(uint64_t seed, uint64_t i, uint64_t len);
uint64_t orc_mixed_len(uint64_t seed, uint64_t i);
void orc_ipv4_tcp_headers(uint64_t seed, uint64_t i, uint64_t dgram_len, uint8_t* dgram);

#ifdef __cplusplus
}
#endif

#endif
