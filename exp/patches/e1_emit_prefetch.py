# gene_emit_staged: the next half's columns loaded before the current half's rank / scan / scatter /
# write phase (software pipelining across the two halves of a tile)
import sys
p = sys.argv[1] + "/gene.h"
s = open(p).read()
old = s[s.index("  for (int h = 0; h < kEmitParts; h++) {\n    const int64_t hb = base + (int64_t)h * kEmitHalf;"):s.index("    __syncthreads();\n    // bucket counts -> staging starts (s_loc), in chunks of kBlock buckets")]
new = '''  EmitInV<kSVec> cur[kEmitPer];
#pragma unroll
  for (int j = 0; j < kEmitPer; j++) cur[j].load<kFull>(gene, r, dflags, base + (j * kBlock + t) * kSVec, n);
#pragma unroll
  for (int h = 0; h < kEmitParts; h++) {
    const int64_t hb = base + (int64_t)h * kEmitHalf;
    uint64_t pv[kEmitPer * kSVec];
    uint32_t br[kEmitPer * kSVec];  // bucket << 12 | rank; ~0u: past n
    EmitInV<kSVec> nxt[kEmitPer];
    if (h + 1 < kEmitParts) {
#pragma unroll
      for (int j = 0; j < kEmitPer; j++)
        nxt[j].load<kFull>(gene, r, dflags, hb + kEmitHalf + (j * kBlock + t) * kSVec, n);
    }
#pragma unroll
    for (int j = 0; j < kEmitPer; j++) {
      const int64_t p0 = hb + (j * kBlock + t) * kSVec;
#pragma unroll
      for (int k = 0; k < kSVec; k++) {
        const int i = j * kSVec + k;
        br[i] = ~0u;
        pv[i] = 0;
        if (kFull || p0 + k < n) {
          const uint32_t gk = (uint32_t)cur[j].g[k];
          const uint32_t bk = gk / kGenesPerBucket;
          const uint32_t f = gene_flags(cur[j].bt[k], cur[j].xf[k], cur[j].df[k]);
          pv[i] = gene_payload8(gk, f, cur[j].ug[k], cur[j].ul[k], cur[j].gg[k], cur[j].gl[k], cur[j].gs[k]);
          br[i] = (bk << 12) | atomicAdd(&s_cnt[bk], 1u);
        }
      }
    }
    if (h + 1 < kEmitParts) {
#pragma unroll
      for (int j = 0; j < kEmitPer; j++) cur[j] = nxt[j];
    }
'''
s = s.replace(old, new)
open(p, "w").write(s)
