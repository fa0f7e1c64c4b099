// Internal (not part of the C-ABI): the DECIMAL plan of a handle (decimal.inc), as heap_snapshot.cpp needs it to write
// and read the DECIMAL(38, s) fields of Flink's heap-layout accumulator rows from the engine's 32-bit piece sums.
#pragma once
#include "../../include/flink_amd.h"

struct FwaDecView {
    int32_t active;                 // 0: the handle has no DECIMAL aggregate (the rest is unset)
    fwa_config icfg;                // the internal configuration: fwa_snapshot / fwa_restore blobs are in its layout
    int32_t umap[FWA_MAX_AGGS];     // user aggregate j -> its internal aggregate (non-DECIMAL), -1 for a DECIMAL one
    int32_t npc[FWA_MAX_AGGS];      // DECIMAL user aggregate j: 2 (int64 input) or 4 (16-byte input) pieces, else 0
    int32_t pc[FWA_MAX_AGGS][4];    // ... the internal SUM(BIGINT) aggregate of each piece
    int32_t cnt[FWA_MAX_AGGS];      // ... the internal aggregate of its (non-NULL) count
};
extern "C" int fwa_dec_view(const fwa_engine* e, FwaDecView* v);
