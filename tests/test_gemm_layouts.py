"""Host model of the N/M-major operand image of native/kernels/gemm_bf16_layouts.hip:
64 k-rows x 256 columns per stage, 8-row groups at a 4224-B stride (128-B pad),
16-B chunk c of row k at c ^ 2(k&3).  Checks that (1) the LDS-DMA pieces
(2 k-rows, lane-linear, fixed per-lane source chunk) build exactly that image,
(2) the ds_read_b64_tr_b16 fragment reads deliver the 16x16x32 MFMA operand
(lane l: column l&15 of the subtile, k = 8(l>>4) + j), (3) the reads are
bank-conflict free per 32-lane half."""
import itertools

TGROUP = 4224


def slot_of(k, chunk):
    return chunk ^ (2 * (k & 3))


def lds_addr(k, chunk):
    return (k >> 3) * TGROUP + (k & 7) * 512 + slot_of(k, chunk) * 16


def dma_image():
    """Simulate the 32 pieces (g = 4p + wave) of one operand stage."""
    img = {}
    for p, wave in itertools.product(range(8), range(4)):
        base = p * TGROUP + wave * 1024                    # M0 of the piece
        for lane in range(64):
            h, slot = lane >> 5, lane & 31
            k = 8 * p + 2 * wave + h                       # k-row the lane loads
            c = slot ^ (2 * ((2 * wave + h) & 3))          # global chunk (lane constant)
            for e in range(8):                             # 8 bf16 of the chunk
                img[base + lane * 16 + 2 * e] = (k, c * 8 + e)
    return img


def test_dma_builds_the_swizzled_image():
    img = dma_image()
    for k in range(64):
        for col in range(256):
            a = lds_addr(k, col // 8) + 2 * (col % 8)
            assert img[a] == (k, col), (k, col)


def tr_addrs(lane, i, ks, r):
    G, i16 = lane >> 4, lane & 15
    q = i16 >> 2
    base_off = G * TGROUP + q * 512 + ((i16 & 3) >> 1) * 16 + 8 * (i16 & 1)
    return base_off + ks * 4 * TGROUP + r * 2048 + ((32 * i) ^ (32 * q))


def test_transposed_reads_give_mfma_operand():
    img = dma_image()
    for i, ks in itertools.product(range(16), range(2)):
        frag = {l: [None] * 8 for l in range(64)}
        for r in range(2):
            for g in range(4):
                lanes = list(range(16 * g, 16 * g + 16))
                # lane 4q+p supplies row q, columns 4p..4p+3; lane x receives column x
                rows = [[img[tr_addrs(lanes[4 * q + p], i, ks, r) + 2 * e] for p in range(4)
                         for e in range(4)] for q in range(4)]
                for x, l in enumerate(lanes):
                    for q in range(4):
                        frag[l][4 * r + q] = rows[q][x]
        for l in range(64):
            for j in range(8):
                assert frag[l][j] == (32 * ks + 8 * (l >> 4) + j, 16 * i + (l & 15)), (i, ks, l, j)


def test_transposed_reads_conflict_free():
    for i, ks, r in itertools.product(range(16), range(2), range(2)):
        for half in (range(0, 32), range(32, 64)):
            banks = []
            for l in half:
                a = tr_addrs(l, i, ks, r)
                banks += [(a // 4) % 64, (a // 4 + 1) % 64]
            assert len(set(banks)) == 64, (i, ks, r)


def test_without_pad_would_conflict():
    # same reads with an unpadded 4096-B group stride: rows k and k+8 collide
    banks = []
    for l in range(32):
        G, i16 = l >> 4, l & 15
        q = i16 >> 2
        a = G * 4096 + q * 512 + ((i16 & 3) >> 1) * 16 + 8 * (i16 & 1) + (0 ^ (32 * q))
        banks += [(a // 4) % 64, (a // 4 + 1) % 64]
    assert len(set(banks)) < 64
