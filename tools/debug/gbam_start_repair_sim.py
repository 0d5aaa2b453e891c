# Experiments: CPU simulation of the device record-start guess (k_guess) and repair (k_walk / k_agree /
# k_fix) on a generated BAM of repeated records (tools/e2e_bench.make_gene_bam).
import sys, struct, zlib
sys.path.insert(0, '/root/repo/tools')
import e2e_bench as E
n = E.make_gene_bam('/tmp/g24.bam', 240000, 20, procs=8)
data = open('/tmp/g24.bam', 'rb').read()
outs = []; O = []; off = 0; u = 0
while off < len(data):
    xlen = struct.unpack_from('<H', data, off + 10)[0]
    bsize = struct.unpack_from('<H', data, off + 12 + xlen - 2)[0] + 1
    blk = zlib.decompress(data[off + 12 + xlen: off + bsize - 8], -15)
    O.append(u); u += len(blk); outs.append(blk); off += bsize
U = b''.join(outs); ulen = len(U)
H = E._header_end(U)
starts = set(); p = H
while p < ulen:
    starts.add(p); p += 4 + struct.unpack_from('<I', U, p)[0]
def u32(p): return struct.unpack_from('<I', U, p)[0]
def plausible(p):
    for j in range(4):
        if p == ulen: return True
        if p + 36 > ulen: return False
        bs = u32(p)
        if bs < 33 or p + 4 + bs > ulen: return False
        d = p + 4
        if struct.unpack_from('<i', U, d)[0] < -1 or struct.unpack_from('<i', U, d + 4)[0] < -1: return False
        lrn = U[d + 8]
        if lrn == 0 or 32 + lrn > bs or U[d + 32 + lrn - 1] != 0: return False
        if any(c < 33 or c > 126 for c in U[d + 32: d + 32 + lrn - 1]): return False
        need = 32 + lrn + 4 * struct.unpack_from('<H', U, d + 12)[0] + (u32(d + 16) + 1) // 2 + u32(d + 16)
        if need > bs: return False
        p = d + bs
    return True
bad = 0
for m in range(1, len(O) - 1):
    if O[m] <= H: continue
    p = O[m]
    while p < ulen and not plausible(p): p += 1
    true = min(s for s in starts if s >= O[m])
    if p != true:
        bad += 1
        if bad < 4: print('member', m, 'guess', p - O[m], 'true', true - O[m])
print('members', len(O), 'bad guesses', bad)

# simulate the device repair (k_walk / k_agree / k_fix)
UNK = -1; BAD = -2
nm = len(O)
Oe = O + [ulen]
mH = 0
while mH + 1 < nm and O[mH + 1] <= H: mH += 1
S = [None] * (nm + 1)
for m in range(nm):
    if m < mH: S[m] = UNK
    elif m == mH: S[m] = H
    else:
        p = O[m]; e = min(ulen, p + (1 << 18)); s = UNK
        while p < e:
            if plausible(p): s = p; break
            p += 1
        S[m] = s
S[nm] = ulen
for rnd in range(100):
    land = [UNK] * (nm + 1)
    for m in range(nm):
        if m < mH or S[m] == UNK: continue
        p = S[m]; end = Oe[m + 1]
        while p < end:
            if p + 4 > ulen: p = BAD; break
            bs = u32(p)
            if p + 4 + bs > ulen: p = BAD; break
            p += 4 + bs
        land[m + 1] = p
    ag = [0] * (nm + 1)
    for m in range(nm + 1):
        ag[m] = 0 if m < mH else (1 if (m == mH or land[m] == S[m]) else 0)
    nbad = 0; newS = list(S)
    for m in range(mH + 1, nm + 1):
        if land[m] == S[m]: continue
        if m < nm and ag[m - 1] and land[m] not in (UNK, BAD): newS[m] = land[m]
        nbad += 1
    S = newS
    print('round', rnd, 'bad', nbad)
    if nbad == 0: break
ok = all(S[m] == min(s for s in starts if s >= O[m]) for m in range(mH + 1, nm) if any(s >= O[m] for s in starts))
print('converged correct:', ok)
