"""Seeded synthetic inputs shaped like the reference's workloads.

Host-side data generation for bench.py and the tests (not on the device path).

No dataset or network exists on either machine: SIFT1M-shaped data are a
clustered mixture with integer values in [0,255] (bvecs semantics,
graphann/loader.go:46-51); graphs are exact kNN graphs (small n) or uniform
random degree-m graphs like private-search.go:54-69 `genRandomGraph`.
"""
import numpy as np


def clustered_vectors(n, d, centers=None, sigma=20.0, seed=0):
    rng = np.random.default_rng(seed)
    k = centers or max(1, min(1000, n // 64))
    c = rng.uniform(0, 255, size=(k, d)).astype(np.float32)
    out = np.empty((n, d), dtype=np.float32)
    step = 1 << 18
    for a in range(0, n, step):
        b = min(n, a + step)
        lab = rng.integers(0, k, size=b - a)
        x = c[lab] + rng.normal(0, sigma, size=(b - a, d)).astype(np.float32)
        out[a:b] = np.clip(np.rint(x), 0, 255)
    return out


def sift_like_vectors(n, d, seed=0, latent=12, centers=64):
    """SIFT1M-shaped stand-in with low intrinsic dimension (real SIFT's is ~10-20):
    a 12-D Gaussian mixture of overlapping clusters, mapped to d dims by a
    random linear map plus noise, scaled per dimension and rounded to integer
    values in [0,255] (bvecs semantics).  Unlike clustered_vectors' isolated
    blobs, its kNN graph is navigable, so recall@10 means something."""
    rng = np.random.default_rng(seed)
    c = rng.normal(0, 2.0, size=(centers, latent))
    W = rng.normal(0, 1.0, size=(latent, d)).astype(np.float32)
    # per-dimension affine scaling from the generating distribution's moments
    mean = c.mean(0) @ W
    var = ((c.var(0) + 1.0)[:, None] * W.astype(np.float64) ** 2).sum(0) + 1.0
    scale = (40.0 / np.sqrt(var)).astype(np.float32)
    out = np.empty((n, d), dtype=np.float32)
    step = 1 << 17
    for a in range(0, n, step):
        b = min(n, a + step)
        z = (c[rng.integers(0, centers, size=b - a)] + rng.normal(0, 1.0, size=(b - a, latent))).astype(np.float32)
        x = z @ W + rng.normal(0, 1.0, size=(b - a, d)).astype(np.float32)
        out[a:b] = np.clip(np.rint((x - mean.astype(np.float32)) * scale + 100.0), 0, 255)
    return out


def knn_graph(v, m):
    """Exact m-NN graph (no self loops) by brute force; small n only."""
    n = v.shape[0]
    sq = (v.astype(np.float64) ** 2).sum(1)
    g = np.empty((n, m), dtype=np.uint32)
    for a in range(0, n, 1024):
        b = min(n, a + 1024)
        d2 = sq[a:b, None] + sq[None, :] - 2.0 * v[a:b].astype(np.float64) @ v.T.astype(np.float64)
        d2[np.arange(b - a), np.arange(a, b)] = np.inf
        g[a:b] = np.argpartition(d2, m, axis=1)[:, :m]
    return g


def random_graph(n, m, seed=0):
    """genRandomGraph (private-search.go:54-69): uniform ids, no self loops."""
    rng = np.random.default_rng(seed)
    g = rng.integers(0, n, size=(n, m), dtype=np.int64)
    self_loop = g == np.arange(n)[:, None]
    while self_loop.any():
        g[self_loop] = rng.integers(0, n, size=int(self_loop.sum()))
        self_loop = g == np.arange(n)[:, None]
    return g.astype(np.uint32)


def msmarco_like_vectors(n, d=192, seed=0, sigma_hi=0.82, sigma_lo=0.29, latent=16, centers=256, block=1 << 17):
    """MS-MARCO-shaped stand-in: the reference's corpus is
    768-d TAS-B embeddings reduced to 192 dims by PCA
    (reproduction/msmarco/embed_and_reduce.py).  Dimension j is centred with
    a standard deviation decaying along the principal axes — 0.82 at j = 0 to
    0.29 at j = d-1 in the reference's validation fixture — and, like real
    embeddings, the points have a low intrinsic dimension (iid Gaussian
    coordinates in 192-d would make every point nearly equidistant from every
    other, and no graph index works on that).  Here: a `latent`-dim Gaussian
    mixture of `centers` overlapping clusters, mapped to d dims by a random
    linear map plus isotropic noise, then every dimension standardised and
    scaled to sigma_j (geometric between the two ends), float32."""
    rng = np.random.default_rng(seed)
    c = rng.normal(0, 1.5, size=(centers, latent))
    W = rng.normal(0, 1.0, size=(latent, d))
    noise = 0.35
    mean = c.mean(0) @ W
    var = ((c.var(0) + 1.0)[:, None] * W ** 2).sum(0) + noise ** 2
    sig = sigma_hi * (sigma_lo / sigma_hi) ** (np.arange(d) / max(1, d - 1))
    scale = (sig / np.sqrt(var)).astype(np.float32)
    W, mean = W.astype(np.float32), mean.astype(np.float32)
    out = np.empty((n, d), dtype=np.float32)
    for a in range(0, n, block):
        b = min(n, a + block)
        z = (c[rng.integers(0, centers, size=b - a)] + rng.normal(0, 1.0, size=(b - a, latent))).astype(np.float32)
        x = z @ W + rng.normal(0, noise, size=(b - a, d)).astype(np.float32)
        out[a:b] = (x - mean) * scale
    return out
