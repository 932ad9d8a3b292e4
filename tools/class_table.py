"""Generates and checks kX6ClassRow (csrc/hz_net.hip), the tower conv's
tap-class row blocks, for bank-conflict-free A-fragment reads: models every
ds_read_b128 of a chunk (lane groups and banks of MI355X_MICROARCH.md's LDS
table, the zero-region redirects of the corner rows, the padding rows' reads)
and prints the LDS-array cycles against the conflict-free count.
Usage: python tools/class_table.py  (exits 1 if the source table differs from
the generated one or has conflicts)"""
import os
import re
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, 'harmonies-alphazero_amd/csrc/hz_net.hip')).read()
m = re.search(r'kX6ClassRow\[18\]\[16\] = \{(.*?)\n\};', src, re.S)
cur = [[int(x) for x in re.findall(r'-?\d+', l.split('//')[0])] for l in m.group(1).strip().split('\n')]
TAPS = [[0x1ff]*4 + [0x1f8, 0x1f8, 0x03f, 0x1b6, 0x0db], [0x1ff]*4 + [0x1f8, 0x03f, 0x03f, 0x1b6, 0x0db]]
SEL = [[0]*9, [0,0,0,0,0x048,0,0x024,0x180,0x003]]
def valid(c):
    ch, cw = divmod(c, 7); v = 0
    for t in range(9):
        hh, ww = ch + t//3 - 1, cw + t%3 - 1
        if 0 <= hh < 5 and 0 <= ww < 7: v |= 1 << t
    return v
G128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128 += [[l+32 for l in g] for g in G128]
CELL, KZERO = 224, 8*35*224
def cyc(addrs):
    tot = 0
    for g in G128:
        slots = {}
        for l in g:
            a = addrs[l]
            slots.setdefault((a % 256)//16, set()).add(a//16)
        tot += max(len(v) for v in slots.values())
    return tot
KPAD = (4*35*224) & ~255
def cost(table, wildcard):
    tot = ideal = 0
    for h in range(2):
        for rb in range(9):
            blk = table[h*9+rb]
            for tap in range(9):
                if not (TAPS[h][rb] >> tap) & 1: continue
                d = ((tap//3-1)*7 + (tap%3-1)) * CELL
                for pa in range(3):
                    addrs = []
                    for lane in range(64):
                        kg = lane >> 4
                        r = blk[lane & 15]
                        if r < 0:
                            if wildcard:
                                cb, v = KPAD + 32*(-1-r) + 16*kg, 0x1ff
                            else:
                                r0 = blk[0]; cb, v = r0*CELL + 16*kg, valid(r0 % 35)
                        else:
                            cb, v = r*CELL + 16*kg, valid(r % 35)
                        a = cb + d
                        if (SEL[h][rb] >> tap) & 1 and not (v >> tap) & 1:
                            a = KZERO + (a & 255)
                        else:
                            assert (v >> tap) & 1, (h, rb, tap, r)
                        addrs.append(a + 64*pa)
                    tot += cyc(addrs); ideal += 4
    return tot, ideal
print('source table (padding as bank wildcards)', cost(cur, True))
# construction
cls = {}
for s in range(8):
    for c in range(35):
        ch, cw = divmod(c, 7)
        k = ('TL' if (ch, cw) == (0, 0) else 'TR' if (ch, cw) == (0, 6) else 'BL' if (ch, cw) == (4, 0) else
             'BR' if (ch, cw) == (4, 6) else 'TM' if ch == 0 else 'BM' if ch == 4 else 'ML' if cw == 0 else
             'MR' if cw == 6 else 'MM')
        cls.setdefault(k, []).append(35*s + c)
def rho(r): return r % 8
def bucket(rows):
    b = {k: [] for k in range(8)}
    for r in rows: b[rho(r)].append(r)
    return b
def arrange(rows):
    """16 rows, each residue twice -> positions S1 gets one, S2 the other."""
    b = bucket(rows)
    assert all(len(v) == 2 for v in b.values()), {k: len(v) for k, v in b.items()}
    S1 = [0,1,2,3,12,13,14,15]; S2 = list(range(4,12))
    out = [None]*16
    for k in range(8):
        x, y = sorted(b[k])
        out[S1[k]] = x; out[S2[k]] = y
    return out
def split(rows, counts):
    """rows -> len(counts) groups; group j takes counts[j] rows of every residue."""
    b = bucket(sorted(rows))
    groups = [[] for _ in counts]
    for k in range(8):
        v = b[k]; assert len(v) == sum(counts), (k, len(v), counts)
        i = 0
        for j, n in enumerate(counts):
            groups[j] += v[i:i+n]; i += n
    return groups
WILD = [-1 - k for k in range(8)]  # padding with residue k
def wild_rows():  # pseudo-rows: residue k; encoded later
    return ['W%d' % k for k in range(8)]
mm = split(cls['MM'], [2]*7 + [1])
tm = split(cls['TM'], [2, 2, 1])
bm = split(cls['BM'], [2, 2, 1])
ml = split(cls['ML'], [2, 1])
mr = split(cls['MR'], [2, 1])
def arr_w(rows, wild):
    # rows: 8 real (one per residue) + 8 others (one per residue) given as rows or wildcard residues
    b = bucket(rows)
    S1 = [0,1,2,3,12,13,14,15]; S2 = list(range(4,12))
    out = [None]*16
    for k in range(8):
        out[S1[k]] = b[k][0]
        out[S2[k]] = (-1 - k) if wild else None
    return out
blocks = [arrange(mm[0]), arrange(mm[1]), arrange(mm[2]), arrange(mm[3]),
          arrange(tm[0]), arrange(tm[1]), arrange(bm[0]), arrange(ml[0]), arrange(mr[0]),
          arrange(mm[4]), arrange(mm[5]), arrange(mm[6])]
# MM block with 8 wildcards
blk = arr_w(mm[7], True); blocks.append(blk)
blocks += [arrange(tm[2] + cls['TL']), arrange(bm[1]), arrange(bm[2] + cls['BR']), arrange(ml[1] + cls['BL']),
           arrange(mr[1] + cls['TR'])]
assert len(blocks) == 18
rows = sorted(r for b in blocks for r in b if r >= 0)
assert rows == list(range(280)), len(rows)
print('new', cost(blocks, True))
names = ['MM']*4 + ['TM', 'TM', 'BM', 'ML', 'MR'] + ['MM']*4 + ['TM+TL', 'BM', 'BM+BR', 'ML+BL', 'MR+TR']
text = ''.join('    {' + ', '.join(str(x) for x in b) + '},  // ' + n + '\n' for b, n in zip(blocks, names))
if '-p' in sys.argv:
    print(text)
def cyc_w64(addrs):  # ds_write_b64: 4 x 16 contiguous lanes, bank (a/4) mod 32
    tot = 0
    for g in range(4):
        banks = {}
        for l in range(16*g, 16*g+16):
            for k in range(2):
                d = addrs[l]//4 + k
                banks.setdefault(d % 32, set()).add(d)
        tot += max(len(v) for v in banks.values())
    return tot
def staging(rowmap):  # k_conv3x3_x6w4's stage_put: 9 float4 per thread, 4 waves, 3 planes
    tot = 0
    for it in range(9):
        for w in range(4):
            for pl in range(3):
                addrs = []
                for lane in range(64):
                    f = min(it*256 + w*64 + lane, 280*8-1)
                    addrs.append(rowmap(f >> 3)*224 + 8*(f & 7) + 64*pl)
                tot += cyc_w64(addrs)
    return tot
srow = lambda r: (r & ~3) | ((r & 1) << 1) | ((r >> 1) & 1)
print('staging stores: rows in order', staging(lambda r: r), ', srow (bits 0, 1 swapped)', staging(srow),
      ', conflict-free', 9*4*3*4)
t, i = cost(blocks, True)
ok = cur == blocks and t == i
print('generated table', (t, i), 'source table equals it' if cur == blocks else 'SOURCE TABLE DIFFERS')
sys.exit(0 if ok else 1)
