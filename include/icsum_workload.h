/*
 * icsum_workload.h — synthetic segment batches for benches and parity tests.
 *
 * These generators live in libicsum.so next to the engine so that a GPU box
 * can build the BASELINE.json workloads directly in HBM (no 1.5-75 GB host
 * transfers).  They implement the seeded splitmix64 spec written out in
 * DESIGN.md §"Workload spec"; oracle/icsum_oracle.c restates the same spec on
 * the CPU and tests/ check the two agree byte for byte.  They are not part of
 * the checksum path.
 */
#ifndef ICSUM_WORKLOAD_H
#define ICSUM_WORKLOAD_H

#include <stdint.h>
#include "icsum.h"

#ifdef __cplusplus
extern "C" {
#endif

/* bytes[j] = spec byte at stream position pos0 + j, j in [0, nbytes). */
int icsw_fill_bytes(ics_ctx* ctx, void* d_bytes, uint64_t nbytes, uint64_t seed,
                    uint64_t pos0, void* stream);

/* d_init[i] = IPv4 pseudo-header sum for segment (index0 + i) of length L_i
 * (seg_len, or d_offsets[i+1]-d_offsets[i]); src/dst from the spec. */
int icsw_pseudo_inits(ics_ctx* ctx, uint32_t* d_init, const uint64_t* d_offsets,
                      uint64_t seg_len, uint64_t n, uint64_t seed, uint64_t index0,
                      void* stream);

/* Overwrite the IPv4 + TCP header fields of n datagrams laid out at `stride`
 * (datagram i = index0 + i, total length dgram_len) per the spec; the payload
 * and the two checksum fields keep the random stream bytes. */
int icsw_ipv4_tcp_headers(ics_ctx* ctx, void* d_dgrams, uint64_t stride, uint64_t dgram_len,
                          uint64_t n, uint64_t seed, uint64_t index0, void* stream);

/* Host-side: mixed-length segment lengths / packed offsets (integer-only
 * log-uniform spec, 64..65535 bytes).  h_offsets has n+1 entries. */
uint64_t icsw_mixed_len(uint64_t seed, uint64_t i);
int icsw_mixed_offsets(uint64_t* h_offsets, uint64_t n, uint64_t seed);

#ifdef __cplusplus
}
#endif

#endif /* ICSUM_WORKLOAD_H */
