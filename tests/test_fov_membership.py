"""The device's FOV queries (k_observe, the greedy policy, the pixel and wide
observations) test Cell.isInFov alone, where the reference's getPelletsInFov /
getEnemyPlayerCellsInFov / getVirusesInFov (field.py:434-456) first query the
spatial hash around the FOV box (spatialHashTable.py:70-83 getIdsForArea,
radius fovSize / 2) and then filter by isInFov (cell.py:169-177).  That is
exact because isInFov implies that the object's bucket footprint meets the
query's (aigar_sem.h, in_fov).  Checked here on the reference's own formulas
(Python floats through numpy: the same IEEE doubles), random and bucket-edge
inputs; parity unpinned only in the sense that no reference run is involved --
both sides are the reference's expressions."""
import numpy as np

B = 20  # HASH_BUCKET_SIZE


def footprint(px, py, rad, size):
    """getIdsForArea as a bucket rectangle [x0, x1] x [y0, y1] (empty: x1 < x0)."""
    def axis(p):
        cl = np.maximum(0.0, p - rad)
        bl = np.floor(cl - np.mod(cl, B))            # int(cellLeft - cellLeft % bucketSize)
        lim = np.floor(np.minimum(size, p + rad + 1))  # int(min(size, pos + radius + 1))
        b0 = np.floor(bl / B)
        b1 = np.where(lim > bl, np.floor((lim - 1 - bl) / B) * B + bl, bl - B)  # last x of range(bl, lim, 20)
        return b0, np.floor(b1 / B)
    x0, x1 = axis(px)
    y0, y1 = axis(py)
    return x0, x1, y0, y1


def in_fov(x, y, r, fx, fy, fs):
    h = fs / 2
    return ~((x + r < fx - h) | (x - r > fx + h) | (y + r < fy - h) | (y - r > fy + h))


def _check(rng, n, size):
    fs = np.concatenate([rng.uniform(10, 450, n // 2), np.full(n - n // 2, rng.uniform(20, 120))])
    fx, fy = rng.uniform(0, size, n), rng.uniform(0, size, n)
    r = np.concatenate([rng.choice([0.5641895835477563, 0.7978845608028654, 0.9772050238058398], n // 2),
                        rng.uniform(0.5, 85, n - n // 2)])
    x = fx + rng.uniform(-1, 1, n) * (fs / 2 + r + 3)
    y = fy + rng.uniform(-1, 1, n) * (fs / 2 + r + 3)
    # bucket-edge and field-edge cases: object edges and FOV edges on multiples of 20, and 0 / size
    k = n // 4
    x[:k] = np.round(x[:k] / B) * B + r[:k] * rng.choice([-1, 1], k)
    y[k:2 * k] = np.round(y[k:2 * k] / B) * B - r[k:2 * k] * rng.choice([-1, 1], k)
    fx[2 * k:3 * k] = np.round((fx[2 * k:3 * k] - fs[2 * k:3 * k] / 2) / B) * B + fs[2 * k:3 * k] / 2
    x[3 * k:3 * k + k // 2] = rng.choice([0.0, float(size)], k // 2)
    for a in (x, y, fx, fy):
        np.clip(a, 0, size, out=a)  # positions live in the field
    vis = in_fov(x, y, r, fx, fy, fs)
    px0, px1, py0, py1 = footprint(x, y, r, size)
    qx0, qx1, qy0, qy1 = footprint(fx, fy, fs / 2, size)
    hit = (px0 <= px1) & (py0 <= py1) & (qx0 <= qx1) & (qy0 <= qy1) & (px0 <= qx1) & (qx0 <= px1) & \
          (py0 <= qy1) & (qy0 <= py1)
    bad = vis & ~hit
    assert not bad.any(), (x[bad][:3], y[bad][:3], r[bad][:3], fx[bad][:3], fy[bad][:3], fs[bad][:3])
    return int(vis.sum())


def test_in_fov_implies_the_hash_query():
    rng = np.random.default_rng(2024)
    seen = 0
    for size in (4800, 1697, 1200, 1000, 500, 250, 4810):
        seen += _check(rng, 300_000, size)
    assert seen > 500_000  # (the check ran on many visible objects)
