/* TEST INFRASTRUCTURE ONLY: exports the reference's own flow hash (dataplane/src/flow/tluhash.h, included
 * unmodified from the reference tree by oracle/Makefile) so the oracle's restatement can be checked against it. */
#include <stdint.h>
#include "tluhash.h"

uint32_t ref_TluHash(uint32_t u1, uint32_t u2) { return TluHash(u1, u2); }

uint32_t ref_flow_hashfn(uint8_t proto, uint32_t sip, uint32_t dip, uint16_t sport, uint16_t dport) {
    return flow_hashfn(proto, sip, dip, sport, dport);
}

void ref_flow_hashfn_batch(const uint32_t *tuple, uint32_t n, uint32_t *out) {
    for (uint32_t i = 0; i < n; i++)
        out[i] = flow_hashfn((uint8_t)tuple[4 * i + 3], tuple[4 * i], tuple[4 * i + 1], (uint16_t)tuple[4 * i + 2],
                             (uint16_t)(tuple[4 * i + 2] >> 16));
}
