"""Host-side estimates behind the shadow bundles / camera lists:
the length of the candidate-leaf lists per 8x8-pixel tile, against the instance-level work of
the reference's own DFS, from the scene file and the reference-identical BVH (no GPU).

    python tools/list_estimates.py [instance10000|instance100k]

* shadow bundles: a tile's floor hit points (rays from the camera to y = 0) swept to each
  light, leaves of the instance tree not separated by the hull's planes
* camera lists: leaves not outside the tile's camera cone
* the reference's instance-level DFS node tests per camera ray (tmax = the oracle's hit
  distance: a lower bound) and, for the entered instances, shape leaves inside the cone vs the
  shape-level DFS node tests (why shape-level lists were not built)
"""
import gzip
import struct
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT)), sys.path.insert(0, str(ROOT / "tests"))
f = np.float32


class Reader:
    def __init__(self, data):
        self.b, self.o = data, 8

    def u32(self):
        v = struct.unpack_from("<I", self.b, self.o)[0]
        self.o += 4
        return v

    def raw(self, n):
        v = self.b[self.o:self.o + n]
        self.o += n
        return v

    def vec(self, dt, k):
        n = self.u32()
        a = np.frombuffer(self.raw(n * np.dtype(dt).itemsize * k), dt)
        return a.reshape(n, k) if k > 1 else a


def load(name):
    import yocto_raytracing_amd as y

    path = ROOT / "tests" / "golden" / "scenes" / f"{name}.yrtscene"
    r = Reader(gzip.open(path).read())
    cams = []
    for _ in range(r.u32()):
        fr = np.frombuffer(r.raw(48), f).reshape(4, 3)
        fovy, aspect, _, focus = struct.unpack("<4f", r.raw(16))
        cams.append((fr, fovy, aspect, focus))
    for _ in range(r.u32()):
        w, h = struct.unpack("<2i", r.raw(8))
        r.raw(w * h * 4)
    mats = []
    for _ in range(r.u32()):
        mats.append(np.frombuffer(r.raw(12), f))
        r.raw(12 * 3 + 4 + 8)
    shapes = []
    for _ in range(r.u32()):
        pos = r.vec(f, 3)
        r.vec(f, 3), r.vec(f, 2), r.vec(f, 1), r.vec(np.int32, 1), r.vec(np.int32, 2), r.vec(np.int32, 3)
        shapes.append(pos)
    insts = []
    for _ in range(r.u32()):
        fr = np.frombuffer(r.raw(48), f).reshape(4, 3)
        s, m = struct.unpack("<2i", r.raw(8))
        insts.append((fr, s, m))
    lights = [(fr[3] + shapes[s][0]).astype(f) for fr, s, m in insts if (mats[m] > 0).all()]
    scn = y.load_scene(str(path))
    y.build_bvh(scn)
    tmp = Path("/tmp") / f"{name}.list_estimates.yrtbvh"
    scn.save_bvh(str(tmp))
    r = Reader(gzip.open(tmp).read())

    def nodes():
        n = r.u32()
        a = np.frombuffer(r.raw(n * 32), np.uint8).reshape(n, 32).copy()
        lp = r.vec(np.int32, 1)
        return (a[:, :24].view(f).reshape(-1, 6), a[:, 24:28].view(np.uint32).ravel(), a[:, 28:30].view(np.uint16).ravel(),
                a[:, 30], lp)

    strees = [nodes() for _ in range(r.u32())]
    return cams[0], lights, insts, strees, nodes()


def planes_hull(P0, P1, L):
    out = []
    for e in range(12):
        a, b, c = e >> 2, ((e >> 2) + 1) % 3, ((e >> 2) + 2) % 3
        bh, ch = e & 1, (e >> 1) & 1
        fb = L[b] > P1[b] if bh else L[b] < P0[b]
        fc = L[c] > P1[c] if ch else L[c] < P0[c]
        if fb == fc:
            continue
        e0, e1 = np.zeros(3, f), np.zeros(3, f)
        e0[a], e1[a] = P0[a], P1[a]
        e0[b] = e1[b] = P1[b] if bh else P0[b]
        e0[c] = e1[c] = P1[c] if ch else P0[c]
        n = np.cross(e1 - e0, L - e0).astype(f)
        if (n * (0.5 * (P0 + P1) - e0)).sum() > 0:
            n = -n
        out.append((n, (n * e0).sum()))
    return out


def outside(boxes, n, d, margin):
    return (np.where(n > 0, boxes[:, :3], boxes[:, 3:]) * n).sum(1) - d > margin


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "instance10000"
    (fr, fovy, aspect, focus), lights, insts, strees, (tb, tstart, tcount, tleaf, tlp) = load(name)
    from helpers import Oracle

    orc = Oracle(name)
    W, H = 1920, 1080
    h = 2 * focus * np.tan(fovy / 2)
    w = h * aspect
    X, Yn, Z, O = fr[0], -fr[1], fr[2], fr[3]

    def dirv(u, v):
        return ((u - 0.5) * w * X + (v - 0.5) * h * Yn - focus * Z).astype(f)

    L = np.where(tleaf == 1)[0]
    lb = tb[L]
    M = max(np.abs(lb).max(), np.abs(O).max())
    eps = 1e-3 + 3e-5 * M
    rng = np.random.default_rng(0)
    shadow, cam, dcounts, sleaves, sdfs = [], [], [], [], []
    for _ in range(200):
        tx, ty = rng.integers(0, W // 8), rng.integers(0, H // 8)
        u0, u1, v0, v1 = tx * 8 / W, (tx * 8 + 8) / W, ty * 8 / H, (ty * 8 + 8) / H
        cu, cv = [u0, u1, u1, u0], [v0, v0, v1, v1]
        c = dirv((u0 + u1) / 2, (v0 + v1) / 2)
        P = []
        for k in range(4):
            n = np.cross(dirv(cu[k], cv[k]), dirv(cu[(k + 1) % 4], cv[(k + 1) % 4]))
            P.append(-n if (n * c).sum() > 0 else n)
        rel = np.concatenate([lb[:, :3] - O, lb[:, 3:] - O], 1)
        m = np.ones(len(lb), bool)
        for n in P:
            m &= ~outside(rel, n, 0.0, np.abs(n).sum() * eps)
        cam.append(m.sum())
        # shadow bundles from the tile's floor points (y = 0)
        d4 = np.array([dirv(u, v) for u, v in zip(cu, cv)])
        t = -O[1] / d4[:, 1]
        if (t > 0).all():
            p = (O + t[:, None] * d4).astype(f)
            P0, P1 = p.min(0), p.max(0)
            for Lp in lights:
                ms = np.all((lb[:, :3] <= np.maximum(P1, Lp) + eps) & (lb[:, 3:] >= np.minimum(P0, Lp) - eps), 1)
                for n, dd in planes_hull(P0, P1, Lp):
                    ms &= ~outside(lb, n, dd, np.abs(n).sum() * (eps + 1e-5 * M))
                shadow.append(ms.sum())
        # the reference's DFS for the tile's centre ray, with the oracle's hit distance as tmax
        dc = c / np.linalg.norm(c)
        hit = orc.trace(np.array([list(O) + list(dc) + [1e-4, 3.4e38]], f))
        tmax = hit["dist"][0] if hit["hit"][0] else np.inf

        def dfs(bb, start, leaf, orig, visit_leaf=None):
            inv, cnt, st = 1 / dc, 0, [0]
            while st:
                x = st.pop()
                cnt += 1
                t0, t1 = (bb[x, :3] - orig) * inv, (bb[x, 3:] - orig) * inv
                if max(np.minimum(t0, t1).max(), 1e-4) > min(np.maximum(t0, t1).min(), tmax) * 1.00000024:
                    continue
                if leaf[x]:
                    if visit_leaf:
                        visit_leaf(x)
                    continue
                st += [start[x], start[x] + 1]
            return cnt

        entered = []
        dfs_n = dfs(tb, tstart, tleaf, O, lambda x: entered.extend(tlp[tstart[x]:tstart[x] + tcount[x]]))
        dcounts.append(dfs_n)
        nl = ns = 0
        for ii in entered:
            ifr, si, _ = insts[ii]
            sb, sst, _, sl, _ = strees[si]
            apex = (O - ifr[3]).astype(f)
            Ls = np.where(sl == 1)[0]
            rels = np.concatenate([sb[Ls, :3] - apex, sb[Ls, 3:] - apex], 1)
            ms = np.ones(len(Ls), bool)
            for n in P:
                ms &= ~outside(rels, n, 0.0, np.abs(n).sum() * eps)
            nl += ms.sum()
            ns += dfs(sb, sst, sl, apex)
        sleaves.append(nl), sdfs.append(ns)
    q = lambda a: f"mean {np.mean(a):.1f} median {np.median(a):.0f} p90 {np.percentile(a, 90):.0f} max {np.max(a)}"
    print(f"{name}: bundle lists (floor tiles, per light) {q(shadow)}")
    print(f"{name}: camera lists {q(cam)}; the reference's instance-level DFS node tests per camera ray {q(dcounts)}")
    print(f"{name}: shape leaves inside the cone of the instances entered {q(sleaves)}; "
          f"shape-level DFS node tests {q(sdfs)}")


if __name__ == "__main__":
    main()
