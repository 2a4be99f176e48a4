/* TEST INFRASTRUCTURE ONLY — drives every oracle entry point on exact-size
 * heap buffers (so ASan sees any read past a datagram or segment) and the
 * threaded batch (so TSan sees its workers), and prints one digest line.
 * Built plain, with ASan+UBSan and with TSan by `make -C oracle check asan
 * tsan`; tests/test_sanitizers.py runs all three and compares their digests. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "icsum_oracle.h"

static uint64_t digest = 1469598103934665603ull; /* FNV-1a over every result */
static void mix(uint64_t v)
{
    for (int i = 0; i < 8; ++i) {
        digest ^= (v >> (8 * i)) & 0xff;
        digest *= 1099511628211ull;
    }
}

int main(void)
{
    const uint64_t seed = 0x10710000ull;
    /* a1-a4: every length 0..300, every init class, split at every point */
    for (uint64_t len = 0; len <= 300; ++len) {
        uint8_t* b = malloc(len ? len : 1);
        orc_fill_bytes(seed, len * 977, len, b);
        const uint32_t inits[] = {0u, 1u, 0xFFFFu, 0x5FFFAu, 0xFFFFFFFFu};
        for (int k = 0; k < 5; ++k) {
            orc_cksum c;
            orc_init(&c, inits[k]);
            orc_add(&c, b, len / 3);
            orc_add(&c, b + len / 3, len - len / 3);
            mix(orc_value(&c));
        }
        free(b);
    }
    /* batch: packed odd offsets, single- and multi-threaded (TSan) */
    enum { N = 4099 };
    uint64_t* off = malloc((N + 1) * sizeof *off);
    off[0] = 0;
    for (uint64_t i = 0; i < N; ++i) off[i + 1] = off[i] + orc_mixed_len(seed + 4, i) % 3001;
    uint8_t* bytes = malloc(off[N] ? off[N] : 1);
    orc_fill_bytes(seed + 4, 0, off[N], bytes);
    uint32_t* init = malloc(N * sizeof *init);
    for (uint64_t i = 0; i < N; ++i) init[i] = orc_pseudo_init(seed + 4, i, off[i + 1] - off[i]);
    uint16_t* o1 = malloc(N * sizeof *o1);
    uint16_t* o8 = malloc(N * sizeof *o8);
    uint32_t* sums = malloc(N * sizeof *sums);
    orc_checksum_batch(bytes, off, 0, 0, init, o1, N);
    if (orc_checksum_batch_mt(bytes, off, 0, 0, init, o8, N, 8) != 0) return 2;
    orc_sum_batch(bytes, off, 0, 0, init, NULL, sums, N);
    for (uint64_t i = 0; i < N; ++i) {
        if (o1[i] != o8[i] || orc_fold(sums[i]) != o1[i]) return 3;
        mix(o1[i]);
    }
    /* a7/a8/a10/a11/a13 + router: datagrams of every length 0..120 and a few
     * MTU ones, exact-size allocations, all three modes */
    for (uint64_t len = 0; len <= 1500; len += (len < 120 ? 1 : 460)) {
        for (int mode = 0; mode < 3; ++mode) {
            uint8_t* d = malloc(len ? len : 1);
            orc_fill_bytes(seed + 2, len * 31 + (uint64_t)mode, len, d);
            if (len >= 40) orc_ipv4_tcp_headers(seed + 2, len, len, d);
            uint16_t ip = 0, tcp = 0;
            uint8_t st = 0;
            orc_ipv4_tcp(d, len, mode, &ip, &tcp, &st);
            mix(ip);
            mix(tcp);
            mix(st);
            orc_router_ttl(d, len, &st);
            mix(st);
            free(d);
        }
    }
    free(off);
    free(bytes);
    free(init);
    free(o1);
    free(o8);
    free(sums);
    printf("oracle-check %016llx\n", (unsigned long long)digest);
    return 0;
}
