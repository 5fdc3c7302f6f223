"""Second, independent restatement of the reference traversal in pure Python
with numpy.float32 scalars (TEST INFRASTRUCTURE ONLY).

Written separately from oracle/vr_oracle.c, from the reference source text
(paths relative to /root/reference/VoxelRaymarcher/src), to catch
transcription errors in the C oracle: the tests run both on the same rays and
demand identical packed pixels.  Slow -- meant for a few hundred rays.

Storage is a sorted array of (region, local key) with the colours plus the
sorted set of non-empty 8^3 clusters; lookups return the same values as
VoxelClusterStore / CuckooHashTable (any correct structure does), and the VCS
existence test is the cluster set (VoxelClusterStore.cuh:93-99).

Algorithmic bytes, counted independently of the C oracle and the GPU
counters: +4 per region-table read (Renderer.cuh:383,408,184,209,...); VCS: +4 per
cluster-existence check (VoxelClusterStore.cuh:93-99; the duplicate directory read of
lookupVoxel, :133, counted once), per lookup +4 for the block's count, +4 per key probe of
performBinarySearch (:101-126, run here over the cluster's sorted keys) and +4 for the
value on a match; cuckoo (CuckooHashTable.cuh:59-76): +4 key1, then +4 val1 on a match
or +4 key2 (+4 val2 on a match) -- which table holds a key is the builder's placement,
passed in (Scene(placement=...)); +4 per pixel write.  Iterations of a crawl run in
closed form are credited +4 each (their existence reads).

No iteration budget.  Walks that the reference never finishes (a loop
iteration that leaves the loop's state unchanged repeats forever) render as
0.  Cluster-skip crawls -- an axis pinned on its skip plane that EPSILON * d
cannot move, so every iteration in the cluster moves the ray by RN(EPSILON *
d) -- are run in closed form with exact rational arithmetic (crawl_run), a
formulation independent of the GPU's float fast-forward (vr_march.hip
crawl_steps) and of the C oracle, which walks them iteration by iteration.
"""
from __future__ import annotations

import math
from fractions import Fraction

import numpy as np

F = np.float32
EPS = F(0.0001)                      # VoxelFunctions.cuh:19
EMPTY = 1 << 30                      # :20-21
CONTINUE = EMPTY + 2                 # :23
INF = F(np.inf)
BLOCK = 64


def f2i(v) -> int:
    """static_cast<int32_t>(float) on the device: truncate, saturate, NaN -> 0."""
    v = float(v)
    if math.isnan(v):
        return 0
    if v >= 2147483648.0:
        return 2147483647
    if v <= -2147483648.0:
        return -2147483648
    return int(v)


def wrap32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def u32(v: int) -> int:
    return v & 0xFFFFFFFF


class V:
    """Vector3f with the reference's operator order (Vector3.cuh)."""
    __slots__ = ("x",)

    def __init__(self, a, b, c):
        self.x = [F(a), F(b), F(c)]

    def __getitem__(self, i):
        return self.x[i]

    def __add__(self, o):
        return V(self.x[0] + o.x[0], self.x[1] + o.x[1], self.x[2] + o.x[2])

    def __sub__(self, o):
        return V(self.x[0] - o.x[0], self.x[1] - o.x[1], self.x[2] - o.x[2])

    def mul(self, o):
        return V(self.x[0] * o.x[0], self.x[1] * o.x[1], self.x[2] * o.x[2])

    def scale(self, t):                  # t * v[i] (Vector3.cuh:130-133, 142-145)
        t = F(t)
        return V(t * self.x[0], t * self.x[1], t * self.x[2])

    def length(self):                    # :79
        return F(np.sqrt(self.x[0] * self.x[0] + self.x[1] * self.x[1] + self.x[2] * self.x[2]))

    def unit(self):                      # :162-165 -> v / length (:136-139)
        n = self.length()
        return V(self.x[0] / n, self.x[1] / n, self.x[2] / n)

    def copy(self):
        return V(*self.x)


def dot(a, b):
    return a.x[0] * b.x[0] + a.x[1] * b.x[1] + a.x[2] * b.x[2]


def cross(a, b):
    return V(a[1] * b[2] - a[2] * b[1], -(a[0] * b[2] - a[2] * b[0]), a[0] * b[1] - a[1] * b[0])


def fmin3(a, b, c):
    return np.fmin(a, np.fmin(b, c))


def same(a, b) -> bool:
    """Loop state equality for the never-finishes test: equal bits, or both NaN."""
    for i in range(3):
        x, y = F(a[i]), F(b[i])
        if not (x.view(np.uint32) == y.view(np.uint32) or (x != x and y != y)):
            return False
    return True


def _rne(q: Fraction) -> int:
    """Round to nearest integer, ties to even."""
    f = q.numerator // q.denominator
    r = q - f
    if r > Fraction(1, 2) or (r == Fraction(1, 2) and f % 2):
        return f + 1
    return f


def crawl_run(p, d, lo):
    """Closed form of a cluster-skip crawl.  p: the position a crawl iteration
    (t = 0 on an axis pinned on its skip plane) produced; every further
    iteration whose start lies in the same cluster [lo_i, lo_i + 8) is the same
    skip, p_i <- RN(p_i + c_i) with c_i = RN(EPSILON * d_i).  Per axis, in units
    of its ulp u: p_i = m u, and RN(m u + c_i) = (m + k) u with k =
    rne(m + c_i / u) - m, constant while p_i stays in its binade (for a tie
    c_i / u = j + 1/2 from the second step on: ties to even keep m even).
    Returns (n, q): n >= 0 iterations whose start positions p, ..., q-step all
    lie in the cluster and whose results q stays in it (n = 0: none), or
    (None, p) when no coordinate moves at all (the crawl never ends)."""
    n = None
    ks = []
    pinned = False
    for i in range(3):
        x = F(p[i])
        c = F(EPS * F(d[i]))
        if not (lo[i] <= float(x) < lo[i] + 8):
            return 0, p
        if F(x + c) == x:                        # the axis never moves
            ks.append(None)
            pinned |= float(d[i]) < 0 and float(x) == lo[i]
            continue
        if not float(x) >= 2.0 ** -100:
            return 0, p
        fr, e = math.frexp(float(x))             # x = fr 2^e, fr in [1/2, 1)
        u = Fraction(2) ** (e - 24)
        m = int(Fraction(float(x)) / u)          # 2^23 <= m < 2^24
        q = Fraction(float(c)) / u
        k0 = _rne(m + q) - m
        k1 = _rne(m + k0 + q) - (m + k0)
        if k0 != k1 or k0 == 0:                   # tie from an odd mantissa: step once more
            return 0, p
        if k0 > 0:
            # every position m + t k (t <= n) below the binade's top and the cluster's
            # upper plane (then every exact sum m + t k + q rounds at spacing u)
            hi_int = min(2 ** 24, (lo[i] + 8) / u) - 1
            na = int((hi_int - m) // k0)
        else:
            # positions at or above the cluster's lower plane, and every exact sum
            # m + t k + q (t < n) at or above the binade's bottom: a sum below it
            # rounds at the finer spacing of the binade beneath
            na = int(min((m - Fraction(lo[i]) / u) // (-k0), (m + q - 2 ** 23) // (-k0) + 1))
        n = na if n is None else min(n, na)
        ks.append((m, k0, u))
    if not pinned:
        return 0, p
    if n is None:
        return None, p
    if n <= 0:
        return 0, p
    out = []
    for i in range(3):
        if ks[i] is None:
            out.append(F(p[i]))
        else:
            m, k, u = ks[i]
            out.append(F(float((m + n * k) * u)))
    return n, V(*out)



class Scene:
    def __init__(self, xyz, rgb, store: int, placement=None):
        """VoxelSceneCPU::insertVoxel (VoxelSceneCPU.cuh:16-46) over the voxels: region =
        floorf(x / 64.0f), local = ((x % 64) + 64) % 64, min/max region coordinate
        scalars starting at 0, later duplicates win (map assignment, :46)."""
        self.store = store
        xyz = np.asarray(xyz, dtype=np.int64).reshape(-1, 3)
        rgb = np.asarray(rgb, dtype=np.int64).reshape(-1)
        r = np.floor(xyz.astype(np.float32) / np.float32(64)).astype(np.int64)
        loc = np.mod(xyz, 64)
        self.min = int(min(0, r.min())) if len(r) else 0
        self.D = (int(max(0, r.max())) if len(r) else 0) - self.min + 1
        rid = self._rid_np(r)
        key = (loc[:, 0] << 20) | (loc[:, 1] << 10) | loc[:, 2]
        comb = (rid << 32) | key
        # the last insertion of a (region, key) wins: first occurrence in the reversed list
        u, first = np.unique(comb[::-1], return_index=True)
        self.keys = u
        self.vals = rgb[::-1][first]
        self.region_ids = np.unique(rid)
        cl = (rid << 9) | ((loc[:, 0] // 8) << 6) | ((loc[:, 1] // 8) << 3) | (loc[:, 2] // 8)
        self.clusters = np.unique(cl)
        # placement(region_index, key) -> 1 or 2: the cuckoo table a stored key sits in
        # (region_index = rank of the region among the occupied ones, the builders' order)
        self.placement = placement
        self._ckeys = {}

    def _rid_np(self, r):
        a = r - self.min
        return a[:, 0] + a[:, 1] * self.D + a[:, 2] * self.D * self.D

    def region_id(self, r):
        a = [v - self.min for v in r]
        rid = a[0] + a[1] * self.D + a[2] * self.D * self.D
        i = np.searchsorted(self.region_ids, rid)
        return rid if i < len(self.region_ids) and self.region_ids[i] == rid else None

    def has_cluster(self, rid, cid):
        c = (rid << 9) | cid
        i = np.searchsorted(self.clusters, c)
        return bool(i < len(self.clusters) and self.clusters[i] == c)

    def get(self, rid, key):
        c = (rid << 32) | key
        i = np.searchsorted(self.keys, c)
        return int(self.vals[i]) if i < len(self.keys) and self.keys[i] == c else EMPTY

    def region_index(self, rid):
        return int(np.searchsorted(self.region_ids, rid))

    def cluster_keys(self, rid, cid):
        """The sorted keys and values of cluster cid of region rid: the block
        [n, (k, v) x n] of VoxelClusterStore.cuh:61-76."""
        got = self._ckeys.get((rid, cid))
        if got is None:
            a, b = np.searchsorted(self.keys, [rid << 32, (rid + 1) << 32])
            k = (self.keys[a:b] & 0xFFFFFFFF).astype(np.int64)
            c = ((k >> 23) << 6) | (((k >> 13) & 7) << 3) | ((k & 0x3FF) >> 3)
            sel = c == cid
            got = ([int(v) for v in k[sel]], [int(v) for v in self.vals[a:b][sel]])
            self._ckeys[(rid, cid)] = got
        return got


class Lighting:
    def __init__(self, shadows=True, point=False, pos=(10.0, 10.0, -10.0)):
        self.L = V(1.0, 1.0, 1.0).unit()      # Main.cu:28
        self.LC = V(1.0, 1.0, 1.0)
        self.LP = V(*pos)
        self.shadows = shadows
        self.point = point


class Walk:
    """One pixel's traversal (Renderer.cuh)."""

    def __init__(self, scene: Scene, lit: Lighting, translation):
        self.s = scene
        self.lit = lit
        self.tr = V(*translation)
        self.iters = 0
        self.bytes = 0
        self.aborted = False

    def tick(self):
        if self.aborted:
            return False
        self.iters += 1
        return True

    def forever(self):
        """The loop would repeat its last iteration forever: the pixel never finishes."""
        self.aborted = True
        return False

    def crawled(self, n):
        """n crawl iterations run in closed form: each one's existence read."""
        self.iters += n
        self.bytes += 4 * n

    # VoxelScene (Renderer.cuh:20-45)
    def in_scene(self, r):
        return all(u32(v - self.s.min) < self.s.D for v in r)

    def region(self, r):
        self.bytes += 4                                  # getRegionStorageStructure's read
        return self.s.region_id(r)

    # StorageStructure adapters (StorageStructure.cuh:24-52)
    def exists(self, reg, x, y, z):
        if self.s.store == 1:
            return True                                  # HashTableStorageStructure: no read
        self.bytes += 4                                  # the directory entry
        ux, uy, uz = u32(x), u32(y), u32(z)
        cid = (((ux // 8) << 6) | ((uy // 8) << 3) | (uz // 8)) & 0xFFFF
        if cid >= 0x8000 or cid >= 512:            # `short` id outside the directory
            return False
        return self.s.has_cluster(reg, cid)

    def lookup(self, reg, x, y, z):
        key = u32((u32(x) << 20) | (u32(y) << 10) | u32(z))
        if self.s.store == 1:
            # CuckooHashTable::lookupVoxel: key1 (+ val1), else key2 (+ val2)
            col = self.s.get(reg, key)
            # (without a placement the bytes of a found key are counted as table 1's)
            table = (self.s.placement(self.s.region_index(reg), key) if self.s.placement else 1) if col != EMPTY else 0
            self.bytes += 8 if table == 1 else (12 if table == 2 else 8)
            return col
        # performBinarySearch over the cluster's sorted keys (only after an existence
        # check: the cluster is in the directory)
        cid = (((u32(x) // 8) << 6) | ((u32(y) // 8) << 3) | (u32(z) // 8)) & 0xFFFF
        keys, vals = self.s.cluster_keys(reg, cid)
        self.bytes += 4                                  # the block's count
        low, high = 0, len(keys) - 1
        while low <= high:
            mid = low + (high - low) // 2
            self.bytes += 4                              # key probe
            if keys[mid] == key:
                self.bytes += 4                          # value
                return vals[mid]
            if keys[mid] < key:
                low = mid + 1
            else:
                high = mid - 1
        return EMPTY

    # lighting (Renderer.cuh:57-86, 249-258; VoxelFunctions.cuh:69-83)
    @staticmethod
    def to_vec(c):
        return V(F(c >> 16) / F(255), F((c >> 8) & 0xFF) / F(255), F(c & 0xFF) / F(255))

    @staticmethod
    def to_int(v):
        ch = [0 if (math.isnan(float(e)) or float(e) <= 0) else int(float(e)) for e in (v[0] * F(255), v[1] * F(255), v[2] * F(255))]
        return (ch[0] << 16) | (ch[1] << 8) | ch[2]

    def lighting(self, color, n, rwp, ro):
        if self.lit.point:
            hp = rwp + ro
            p2l = self.lit.LP - hp
            dist = p2l.length()
            ld = p2l.unit()
            att = F(1) / (F(1.0) + F(0.045) * dist + F(0.0075) * (dist * dist))
            diff = np.fmax(dot(n, ld), F(0))
            diffuse = self.lit.LC.scale(diff)
            return self.to_int(diffuse.scale(att).mul(self.to_vec(color)))
        diff = np.fmax(dot(n, self.lit.L), F(0))
        diffuse = self.lit.LC.scale(diff)
        return self.to_int(self.to_vec(color).mul(diffuse))

    @staticmethod
    def normal(tX, tY, tZ, tMin, d):        # Renderer.cuh:237-247
        if tX == tMin:
            return V(np.copysign(F(1), -d[0]), 0, 0)
        if tY == tMin:
            return V(0, np.copysign(F(1), -d[1]), 0)
        return V(0, 0, np.copysign(F(1), -d[2]))

    @staticmethod
    def nxt(pos, x):                         # Renderer.cuh:47-55
        return F(np.ceil(x)) + EPS if pos else F(np.floor(x)) - EPS

    @staticmethod
    def in_region(o):
        return all(F(0) <= o[i] < F(BLOCK) for i in range(3))

    @staticmethod
    def grid_in(a, b, c):
        return all(u32(v) < BLOCK for v in (a, b, c))

    @staticmethod
    def div(a, b, guard=False):
        a, b = F(a), F(b)
        if guard and b == 0:
            return INF
        with np.errstate(divide="ignore", invalid="ignore"):
            return F(a / b)

    def shift_region(self, cr, o):
        d = [f2i(np.floor(o[i] / F(BLOCK))) for i in range(3)]
        for i in range(3):
            cr[i] = wrap32(cr[i] + d[i])
        return (o - V(wrap32(d[0] * BLOCK), wrap32(d[1] * BLOCK), wrap32(d[2] * BLOCK))).scale(1.0)

    # rayMarchVoxelGrid (:260-336) / shadowRayMarchVoxelGrid (:100-172)
    def grid(self, ray, reg, rwp, cr, shadow):
        o, d = ray[0], ray[1]
        pos = [d[i] > 0 for i in range(3)]
        t = [self.div(self.nxt(pos[i], o[i]) - o[i], d[i], shadow) for i in range(3)]
        tMin = fmin3(*t)
        ray[0] = o + d.scale(tMin + EPS)
        while self.in_region(ray[0]):
            if not self.tick():
                return EMPTY
            o = ray[0]
            vx, vy, vz = (f2i(o[i]) for i in range(3))
            if not self.exists(reg, vx, vy, vz):
                nb = []
                for i, vv in enumerate((vx, vy, vz)):
                    q = int(vv / 8)      # C truncating division
                    nb.append((q + 1) * 8 if pos[i] else q * 8)
                st = [self.div(F(nb[i]) - o[i], d[i], shadow) for i in range(3)]
                smin = fmin3(*st)
                ray[0] = o + d.scale(smin + EPS)
                if same(ray[0], o):
                    self.forever()
                    return EMPTY
                if smin == 0:                    # a crawl: the identical iterations after it at once
                    n, ray[0] = crawl_run(ray[0], d, [(v // 8) * 8 for v in (vx, vy, vz)])
                    if n is None:
                        self.forever()
                        return EMPTY
                    self.crawled(n)
                continue
            col = self.lookup(reg, vx, vy, vz)
            if col != EMPTY:
                if shadow:
                    return col
                lit = self.lighting(col, self.normal(t[0], t[1], t[2], tMin, d), rwp, o)
                return lit * (0 if self.shadow_scene([o.copy(), self.lit.L], list(cr), False) else 1)
            t = [self.div(self.nxt(pos[i], o[i]) - o[i], d[i], shadow) for i in range(3)]
            tMin = fmin3(*t)
            ray[0] = o + d.scale(tMin + EPS)
            if same(ray[0], o):
                self.forever()
                return EMPTY
        return EMPTY

    def null_skip(self, lr, cr, guard):       # :386-409 / :187-210
        o, d = lr[0], lr[1]
        n = [F(BLOCK) + EPS if d[i] > 0 else F(0) - EPS for i in range(3)]
        t = [self.div(n[i] - o[i], d[i], guard) for i in range(3)]
        lr[0] = self.shift_region(cr, o + d.scale(fmin3(*t)))

    # isInShadowOriginalRayMarch (:174-235) / ...LongestAxis (:633-694)
    def shadow_scene(self, lr, cr, longest):
        if not self.lit.shadows:
            return False
        while self.in_scene(cr):
            if not self.tick():
                return False
            cr0, o0 = list(cr), lr[0]
            reg = self.region(cr)
            while reg is None:
                if not self.tick():
                    return False
                cr1, o1 = list(cr), lr[0]
                self.null_skip(lr, cr, not longest)
                if not self.in_scene(cr):
                    return False
                if cr == cr1 and same(lr[0], o1):
                    return self.forever()
                reg = self.region(cr)
            col = self.grid_la(lr, reg, V(0, 0, 0), cr, True) if longest else self.grid(lr, reg, None, cr, True)
            if self.aborted:
                return False
            if col != EMPTY:
                return True
            lr[0] = self.shift_region(cr, lr[0])
            if cr == cr0 and same(lr[0], o0):
                return self.forever()
        return False

    # rayMarchVoxelGridLongestAxis (:760-915) / shadow twin (:495-631)
    def grid_la(self, orig, reg, rwp, cr, shadow):
        od = orig[1]
        a = [abs(od[i]) for i in range(3)]
        if a[0] > a[1] and a[0] > a[2]:
            L, (M, S), k = 0, ((1, 2) if a[1] > a[2] else (2, 1)), F(1) / a[0]
        elif a[1] > a[2]:
            L, (M, S), k = 1, ((0, 2) if a[0] > a[2] else (2, 0)), F(1) / a[1]
        else:
            L, (M, S), k = 2, ((0, 1) if a[0] > a[1] else (1, 0)), F(1) / a[2]
        ds = od.scale(k)
        old = orig[0].copy()
        g = [f2i(orig[0][i]) for i in range(3)]
        ad = [0, 0, 0]
        ad[L] = -1 if od[L] < 0 else 1
        if ad[L] > 0:
            t = (F(g[L]) + EPS + F(1) - orig[0][L]) / F(ad[L])
        else:
            t = (F(g[L]) - EPS - orig[0][L]) / F(ad[L])
        ray = old + ds.scale(t)
        ad[M] = wrap32(f2i(ray[M]) - g[M])
        ad[S] = wrap32(f2i(ray[S]) - g[S])
        floor_mid = ds[M] < 0
        st = {"old": old, "ray": ray}

        def hit(col, axis, loc):
            if shadow:
                return col
            n = [F(0)] * 3
            n[axis] = np.copysign(F(1), -ds[axis])
            lit = self.lighting(col, V(*n), rwp, loc)
            return lit * (0 if self.shadow_scene([loc.copy(), self.lit.L], list(cr), True) else 1)

        def jump():                          # performVoxelSpaceJump (:696-751) / (:441-492)
            tX = tY = tZ = tMin = F(0)
            while not self.exists(reg, *g):
                if not self.tick():
                    return EMPTY
                o = st["old"]
                nb = []
                for i in range(3):
                    q = int(g[i] / 8)
                    nb.append((q + 1) * 8 if ds[i] > 0 else q * 8)
                tX, tY, tZ = (self.div(F(nb[i]) - o[i], ds[i]) for i in range(3))
                tm0 = fmin3(tX, tY, tZ)
                tMin = tm0 + EPS
                st["old"] = o + ds.scale(tMin)
                g0 = list(g)
                for i in range(3):
                    g[i] = f2i(np.floor(st["old"][i]))
                if not self.grid_in(*g):
                    orig[0] = st["old"].copy()
                    return EMPTY
                if same(st["old"], o) and g == g0:
                    self.forever()
                    return EMPTY
                if tm0 == 0:                     # a crawl (as in grid): closed form
                    n, st["old"] = crawl_run(st["old"], ds, [(v // 8) * 8 for v in g0])
                    if n is None:
                        self.forever()
                        return EMPTY
                    self.crawled(n)
                    for i in range(3):
                        g[i] = f2i(np.floor(st["old"][i]))
            col = self.lookup(reg, *g)
            if col != EMPTY:
                if shadow:
                    return col
                lit = self.lighting(col, self.normal(tX, tY, tZ, tMin, ds), rwp, st["old"])
                return lit * (0 if self.shadow_scene([st["old"].copy(), self.lit.L], list(cr), True) else 1)
            o = st["old"]
            if ds[L] > 0:
                tn = (F(np.ceil(o[L])) - o[L]) / ds[L]
            else:
                tn = (F(np.floor(o[L])) - o[L]) / ds[L]
            st["ray"] = o + ds.scale(tn + EPS)
            ad[M] = wrap32(f2i(st["ray"][M]) - g[M])
            ad[S] = wrap32(f2i(st["ray"][S]) - g[S])
            return CONTINUE

        def step(axis, long_axis):
            """-> ('ret', value) | ('cont',) | None"""
            g[axis] = wrap32(g[axis] + ad[axis])
            if not self.exists(reg, *g):
                r = jump()
                if self.aborted:
                    return ("ret", EMPTY)
                return ("ret", r) if r != CONTINUE else ("cont",)
            col = self.lookup(reg, *g)
            if col != EMPTY:
                if long_axis:
                    loc = st["ray"]
                else:                        # getLocalHitLocation (:753-758)
                    o = st["old"]
                    if ds[axis] > 0:
                        tt = (F(np.ceil(o[axis])) - o[axis]) / ds[axis]
                    else:
                        tt = (F(np.floor(o[axis])) - o[axis]) / ds[axis]
                    loc = o + ds.scale(tt)
                return ("ret", hit(col, axis, loc))
            return None

        while self.grid_in(wrap32(g[L] + ad[L]), wrap32(g[M] + ad[M]), wrap32(g[S] + ad[S])):
            if not self.tick():
                return EMPTY
            if ad[S] != 0 and ad[M] != 0:
                om = st["old"][M]
                t1 = ((F(np.floor(om)) if floor_mid else F(np.ceil(om))) - om) / ds[M]
                sp = st["old"][S] + ds[S] * t1
                sd = wrap32(f2i(np.floor(sp)) - g[S])
                order = [S, M] if sd != 0 else [M, S]
            elif ad[M] != 0:
                order = [M]
            elif ad[S] != 0:
                order = [S]
            else:
                order = []
            res = None
            for axis in order + [L]:
                res = step(axis, axis == L)
                if res is not None:
                    break
            if res is not None:
                if res[0] == "ret":
                    return res[1]
                continue
            st["old"] = st["ray"]
            st["ray"] = st["ray"] + ds
            ad[M] = wrap32(f2i(st["ray"][M]) - g[M])
            ad[S] = wrap32(f2i(st["ray"][S]) - g[S])
        orig[0] = st["old"].copy()
        return self.grid(orig, reg, rwp, cr, shadow)

    # rayMarchVoxelScene (:338-434) / rayMarchVoxelSceneLongestAxis (:917-1010)
    def scene(self, world_o, world_d, scale, longest):
        so = (world_o - self.tr).scale(F(scale))
        d = world_d
        cr = [f2i(np.floor(so[i] / F(BLOCK))) for i in range(3)]
        while not self.in_scene(cr):
            if not self.tick():
                return 0
            cr0, o0 = list(cr), so
            hi = wrap32(self.s.D + self.s.min)
            lo = self.s.min
            t = []
            for i in range(3):
                n = hi if d[i] < 0 else lo
                tv = self.div(F(wrap32(n * BLOCK)) - so[i], d[i])
                t.append(INF if tv <= 0 else tv)
            tMin = fmin3(*t)
            if tMin == INF:
                return 0
            so = so + d.scale(tMin + EPS)
            cr = [f2i(np.floor(so[i] / F(BLOCK))) for i in range(3)]
            if cr == cr0 and same(so, o0):
                self.forever()
                return 0
        lr = [(so - V(wrap32(cr[0] * BLOCK), wrap32(cr[1] * BLOCK), wrap32(cr[2] * BLOCK))).scale(1.0), d]
        while self.in_scene(cr):
            if not self.tick():
                return 0
            cr0, o0 = list(cr), lr[0]
            reg = self.region(cr)
            while reg is None:
                if not self.tick():
                    return 0
                cr1, o1 = list(cr), lr[0]
                self.null_skip(lr, cr, False)
                if not self.in_scene(cr):
                    return 0
                if cr == cr1 and same(lr[0], o1):
                    self.forever()
                    return 0
                reg = self.region(cr)
            rwp = self.tr + V(wrap32(cr[0] * BLOCK), wrap32(cr[1] * BLOCK), wrap32(cr[2] * BLOCK))
            col = self.grid_la(lr, reg, rwp, cr, False) if longest else self.grid(lr, reg, rwp, cr, False)
            if self.aborted:
                return 0
            if col != EMPTY:
                return col
            lr[0] = self.shift_region(cr, lr[0])
            if cr == cr0 and same(lr[0], o0):
                self.forever()
                return 0
        return 0


def camera(eye, at, up, fov, aspect):
    """Camera::Camera (Camera.cuh:11-23) -> (origin, llc, horizontal, vertical)."""
    PI = F(3.141592)
    hh = F(math.tan(float((F(fov) * PI / F(180)) / F(2))))
    # tanf: take the float32 rounding of the double tan of the float32 argument
    hw = hh * F(aspect)
    o = V(*eye)
    w = (V(*at) - o).unit()
    u = cross(w, V(*up)).unit()
    v = cross(u, w)
    llc = ((o - u.scale(hw)) - v.scale(hh)) + w
    return o, llc, u.scale(F(2) * hw), v.scale(F(2) * hh)


def render_pixel(scene, lit, cam_fields, W, H, x, y, scale, longest, translation=(0.0, 0.0, 0.0), iters=False,
                 nbytes=False):
    """calculateWorldRay + kernel body (Renderer.cuh:1013-1063). cam_fields: (origin, llc, hor, ver) V's.
    iters: return (colour, loop iterations of the pixel, crawl iterations included);
    nbytes: return (colour, algorithmic bytes of the pixel: its walks' reads + the 4-B pixel write;
    4 alone for a walk that never finishes)."""
    org, llc, hor, ver = cam_fields
    u = (F(x) + F(0.5)) / F(W)
    v = (F(u32(H - y)) + F(0.5)) / F(H)
    ro = (llc + hor.scale(u)) + ver.scale(v)
    rd = (ro - org).unit()
    w = Walk(scene, lit, translation)
    col = w.scene(ro, rd, scale, longest)
    col = 0 if w.aborted else col
    if nbytes:
        return col, (4 if w.aborted else w.bytes + 4)
    return (col, w.iters) if iters else col
