"""Exhaustive search for XOR-linear 16-byte-chunk swizzles of the LDS images of
ks.h / kx.h under which the kernels' ds_read_b128 (lane groups of
MI355X_MICROARCH.md §LDS) and ds_read_b64_tr_b16 (32-lane halves) are bank-conflict
free.  Prints the first map found per image."""
import itertools
G = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G += [[l+32 for l in g] for g in G]
def f_of(M, r):
    v = 0
    for b in range(5):
        if (r >> b) & 1: v ^= M[b]
    return v
def ok_x(M, NCH=16):
    f = lambda r: f_of(M, r)
    # P1 row reads: lane l -> row i*16 + (l&15), chunk c + (l>>4), c multiple of 4
    for i in (0, 1):
        for c in range(0, NCH, 4):
            for g in G:
                s = {((c + (l >> 4)) ^ f(i * 16 + (l & 15))) % 16 for l in g}
                if len(s) != 16: return False
    # gW0 tr reads: lanes 0-31 / 32-63: row 8q+4h+(i>>2), chunk c0 + ((i&3)>>1), c0 even
    for h in (0, 1):
        for c0 in range(0, NCH, 2):
            for half in (0, 1):
                slots = set()
                for l in range(32 * half, 32 * half + 32):
                    q, i = l >> 4, l & 15
                    r = 8 * q + 4 * h + (i >> 2)
                    slots.add((((c0 + ((i & 3) >> 1)) ^ f(r)) % 16, (i & 1)))
                if len(slots) != 32: return False
    return True
for M in itertools.product(range(16), repeat=5):
    if ok_x(M):
        print("xhat swizzle M =", M, [f_of(M, r) for r in range(32)]); break
else:
    print("none (xhat)")

def f_lin(M, r, nb):
    v = 0
    for b in range(nb):
        if (r >> b) & 1: v ^= M[b]
    return v
def ok_w(M):
    f = lambda r: f_lin(M, r, 6)
    # (a) b128 row reads, rows jb*16 + (l&15), chunk 4s + q
    for jb in range(4):
        for s in range(2):
            for g in G:
                pos = {((jb*16 + (l & 15)) & 1) * 8 + (((4 * s + (l >> 4)) ^ f(jb*16 + (l & 15))) % 8) for l in g}
                if len(pos) != 16: return False
    # (b) tr reads rows 32s + 8q + 4h + (i>>2), chunk 2hb + ((i&3)>>1), half i&1
    for s in range(2):
        for h in range(2):
            for hb in range(4):
                for half in range(2):
                    sl = set()
                    for l in range(32 * half, 32 * half + 32):
                        q, i = l >> 4, l & 15
                        r = 32 * s + 8 * q + 4 * h + (i >> 2)
                        if r >= 64: r -= 32
                        sl.add(((r & 1) * 8 + (((2 * hb + ((i & 3) >> 1)) ^ f(r)) % 8), i & 1))
                    if len(sl) != 32: return False
    return True
for M in itertools.product(range(8), repeat=6):
    if ok_w(M):
        print("weight swizzle M =", M, [f_lin(M, r, 6) for r in range(16)]); break
else:
    print("none (weights)")

def ok_a(M):
    g = lambda f: f_lin(M, f, 6)
    # (c) tr: image row f = 32s + 8q + 4h + (i>>2), chunk 2rb + ((i&3)>>1), half
    for s in range(2):
        for h in range(2):
            for rb in range(2):
                for half in range(2):
                    sl = set()
                    for l in range(32 * half, 32 * half + 32):
                        q, i = l >> 4, l & 15
                        f = 32 * s + 8 * q + 4 * h + (i >> 2)
                        sl.add(((f & 3) * 4 + (((2 * rb + ((i & 3) >> 1)) ^ g(f)) % 4), i & 1))
                    if len(sl) != 32: return False
    # (d) b128: image row f = fb*16 + (l&15), chunk q
    for fb in range(4):
        for gg in G:
            pos = {((fb * 16 + (l & 15)) & 3) * 4 + (((l >> 4) ^ g(fb * 16 + (l & 15))) % 4) for l in gg}
            if len(pos) != 16: return False
    return True
for M in itertools.product(range(4), repeat=6):
    if ok_a(M):
        print("act swizzle M =", M, [f_lin(M, r, 6) for r in range(16)]); break
else:
    print("none (act)")
