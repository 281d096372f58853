"""Host model of the LDS image used by native/kernels/attention.hip: 256-B
rows (128 bf16 of one key), 16-B chunk c of row r stored at
c ^ ((r&3)<<2 | (r>>2)&3).  Checks that the K row reads (ds_read_b128, the
A operand of the 32x32x16 S^T = K.Q^T MFMA) and the V transposed reads
(ds_read_b64_tr_b16, the A operand of O^T += V^T.P^T) are bank-conflict
free, and that the transposed read delivers exactly V^T with the k order the
P^T accumulator fragment implies."""
import itertools

B128_GROUPS = [
    list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
    list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
    list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
    list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64)),
]


def swz(row, ch):
    return row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4)


def banks(addr, nbytes):
    return {((addr + 4 * i) // 4) % 64 for i in range(nbytes // 4)}


def test_k_row_reads_conflict_free():
    for kb in range(2):
        for s in range(8):
            for g in B128_GROUPS:
                used = []
                for l in g:
                    used += list(banks(swz(32 * kb + (l & 31), 2 * s + (l >> 5)), 16))
                assert len(used) == len(set(used)) == 64, (kb, s)


def tr_addr(lane, db, ks, jh):
    h, G, i = lane >> 5, lane >> 4, lane & 15
    key = 16 * ks + 8 * jh + 4 * h + (i >> 2)
    ch = 4 * db + 2 * (G & 1) + ((i & 3) >> 1)
    return swz(key, ch) + 8 * (i & 1), key, 32 * db + 16 * (G & 1) + 4 * (i & 3)


def test_v_transposed_reads_conflict_free():
    for db, ks, jh in itertools.product(range(4), range(4), range(2)):
        for half in (range(0, 32), range(32, 64)):
            used = []
            for l in half:
                used += list(banks(tr_addr(l, db, ks, jh)[0], 8))
            assert len(used) == len(set(used)) == 64, (db, ks, jh)


def test_v_transposed_read_semantics():
    """Simulate ds_read_b64_tr_b16 on the swizzled image of V[key][d] = (key, d)
    and check lane l element j == V[key(j, h)][d = 32db + (l & 31)] with the
    permuted key order of the P^T fragment: 16ks + 8(j>>2) + 4h + (j&3)."""
    image = {}
    for key in range(64):
        for d in range(128):
            ch, w = d // 8, d % 8
            image[swz(key, ch) + 2 * w] = (key, d)
    for db, ks in itertools.product(range(4), range(4)):
        frag = {l: [None] * 8 for l in range(64)}
        for jh in range(2):
            addrs = {l: tr_addr(l, db, ks, jh)[0] for l in range(64)}
            for g in range(4):
                lanes = list(range(16 * g, 16 * g + 16))
                # lane 4q+p supplies row q, cols 4p..4p+3; lane i receives column i of the 4 rows
                rows = [[image[addrs[lanes[4 * q + p]] + 2 * e] for p in range(4) for e in range(4)]
                        for q in range(4)]
                for i, l in enumerate(lanes):
                    for q in range(4):
                        frag[l][4 * jh + q] = rows[q][i]
        for l in range(64):
            h = l >> 5
            for j in range(8):
                want = (16 * ks + 8 * (j >> 2) + 4 * h + (j & 3), 32 * db + (l & 31))
                assert frag[l][j] == want, (db, ks, l, j, frag[l][j], want)


# ---- dK/dV kernel (16x16x32 MFMAs): Q / dO image, chunk c of row r at c ^ 2(r&7)
def swz16(row, ch):
    return row * 256 + ((ch ^ (2 * (row & 7))) << 4)


def test_dkdv16_row_reads_conflict_free():
    # A operand of S = Q.K^T: lane l reads row 16t + (l&15), chunk 4s + (l>>4)
    for t in range(4):
        for s in range(4):
            for g in B128_GROUPS:
                used = []
                for l in g:
                    used += list(banks(swz16(16 * t + (l & 15), 4 * s + (l >> 4)), 16))
                assert len(used) == len(set(used)) == 64, (t, s)


def tr16_addr(lane, ks, jh, db):
    G, i = lane >> 4, lane & 15
    row = 32 * ks + 16 * jh + 4 * G + (i >> 2)
    ch = 2 * db + ((i & 3) >> 1)
    return swz16(row, ch) + 8 * (i & 1)


def test_dkdv16_transposed_reads_conflict_free_and_exact():
    image = {}
    for q in range(64):
        for d in range(128):
            image[swz16(q, d // 8) + 2 * (d % 8)] = (q, d)
    for ks, db in itertools.product(range(2), range(8)):
        for jh in range(2):
            for half in (range(0, 32), range(32, 64)):
                used = []
                for l in half:
                    used += list(banks(tr16_addr(l, ks, jh, db), 8))
                assert len(used) == len(set(used)) == 64, (ks, jh, db)
        # semantics: lane l element j = dO[q(j)][d = 16 db + (l & 15)] with the
        # P-fragment query order q(j) = 32 ks + 16 (j >> 2) + 4 (l >> 4) + (j & 3)
        frag = {l: [None] * 8 for l in range(64)}
        for jh in range(2):
            for g in range(4):
                lanes = list(range(16 * g, 16 * g + 16))
                rows = [[image[tr16_addr(lanes[4 * qq + p], ks, jh, db) + 2 * e]
                         for p in range(4) for e in range(4)] for qq in range(4)]
                for x, l in enumerate(lanes):
                    for qq in range(4):
                        frag[l][4 * jh + qq] = rows[qq][x]
        for l in range(64):
            for j in range(8):
                want = (32 * ks + 16 * (j >> 2) + 4 * (l >> 4) + (j & 3), 16 * db + (l & 15))
                assert frag[l][j] == want
