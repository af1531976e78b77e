"""Seeded synthetic matrices of SURVEY.md §8(d) (benchmark and parity inputs).

* ``band``    — k distinct columns per row inside a (2w+1)-wide window around the diagonal,
                values U(-1, 1), one planted diagonal spike A(s, s) = 10 at s = n_global // 2 so the
                dominant eigenvalue is well separated.  Locality-preserving: row blocks only need a
                halo of w entries from their neighbours (the multi-GPU headline, §8e).
* ``uniform`` — k distinct columns uniform over [0, n), values U(0, 1] (nonnegative: Perron root
                ≈ k/2).  The gather-stress case.
* ``triu_complex`` — config 5: complex upper-triangular CSR with an explicit diagonal whose
                entries lie in the annulus 1 <= |z| <= 2, one planted interior eigenvalue
                d* = 1.5 e^{0.7i} isolated by 0.05 (the eigenvalues are the diagonal).

All generators return CSR arrays (rowptr int32, colidx int32 sorted per row, values) for rows
[row0, row0 + nrows) of an n_global x n_global matrix.  band / uniform / start_vector draw their
random numbers in fixed chunks of CHUNK rows seeded by the chunk index, so any row block is
bitwise the same rows of the unsplit matrix (BASELINE config 4 is one 10M matrix split over the
ranks: the N-rank matrix is the N = 1 matrix).
"""
from __future__ import annotations

import numpy as np


def _distinct_sorted(rng, nrows: int, k: int, span: int) -> np.ndarray:
    """k strictly increasing integers in [0, span) per row (sorted-sample + arange trick)."""
    r = rng.integers(0, span - k + 1, size=(nrows, k), dtype=np.int64)
    r.sort(axis=1)
    r += np.arange(k, dtype=np.int64)[None, :]
    return r


CHUNK = 1 << 16   # rows per generator chunk: chunk c is drawn from default_rng([seed, c, tag])


def _chunks(row0: int, nrows: int):
    """(chunk index, first row of the chunk, rows [a, b) of the request inside it)."""
    c0, c1 = row0 // CHUNK, (row0 + nrows + CHUNK - 1) // CHUNK
    for c in range(c0, c1):
        base = c * CHUNK
        yield c, base, max(row0, base), min(row0 + nrows, base + CHUNK)


def band(n_global: int, k: int, w: int = 64, seed: int = 42, row0: int = 0, nrows: int | None = None,
         spike: float = 10.0):
    """Rows [row0, row0 + nrows) of the band matrix.  Partition-invariant: rows are generated in
    fixed chunks of CHUNK rows seeded by the chunk index, so the rows of any row block are bitwise
    the rows of the whole matrix (a matrix split over N ranks is the N = 1 matrix)."""
    if nrows is None:
        nrows = n_global - row0
    width = 2 * w + 1
    if n_global < width or k > width:
        raise ValueError("band: n_global must be >= 2w+1 and k <= 2w+1")
    cols = np.empty((nrows, k), dtype=np.int64)
    vals = np.empty((nrows, k), dtype=np.float64)
    for c, base, a, b in _chunks(row0, nrows):
        m = min(CHUNK, n_global - base)
        rng = np.random.default_rng([seed, c, 0])
        rows = np.arange(base, base + m, dtype=np.int64)
        start = np.clip(rows - w, 0, n_global - width)
        cc = start[:, None] + _distinct_sorted(rng, m, k, width)
        vv = rng.uniform(-1.0, 1.0, size=(m, k))
        cols[a - row0:b - row0] = cc[a - base:b - base]
        vals[a - row0:b - row0] = vv[a - base:b - base]
    s = n_global // 2
    if row0 <= s < row0 + nrows:
        i = s - row0
        c0 = min(max(s - k // 2, 0), n_global - k)
        cols[i] = np.arange(c0, c0 + k)
        vals[i] = 0.0
        vals[i, :] = np.random.default_rng([seed, s, 2]).uniform(-1.0, 1.0, size=k)
        vals[i, s - c0] = spike
    rowptr = np.arange(0, (nrows + 1) * k, k, dtype=np.int64)
    return rowptr.astype(np.int32), cols.reshape(-1).astype(np.int32), vals.reshape(-1)


def uniform(n_global: int, k: int, seed: int = 42, row0: int = 0, nrows: int | None = None):
    """Rows [row0, row0 + nrows) of the uniform-column matrix (partition-invariant, see band)."""
    if nrows is None:
        nrows = n_global - row0
    cols = np.empty((nrows, k), dtype=np.int64)
    vals = np.empty((nrows, k), dtype=np.float64)
    for c, base, a, b in _chunks(row0, nrows):
        m = min(CHUNK, n_global - base)
        rng = np.random.default_rng([seed, c, 1])
        cc = _distinct_sorted(rng, m, k, n_global)
        vv = 1.0 - rng.random(size=(m, k))   # (0, 1]
        cols[a - row0:b - row0] = cc[a - base:b - base]
        vals[a - row0:b - row0] = vv[a - base:b - base]
    rowptr = np.arange(0, (nrows + 1) * k, k, dtype=np.int64)
    return rowptr.astype(np.int32), cols.reshape(-1).astype(np.int32), vals.reshape(-1)


def triu_complex(n: int, k: int, seed: int = 42, target=1.5 * np.exp(0.7j), gap: float = 0.05):
    """Upper-triangular complex CSR, k nonzeros per row including the diagonal (config 5).

    Returns (rowptr, colidx, values, diagonal); the eigenvalues are the diagonal, with the target
    planted at row n // 3 and no other diagonal entry within `gap` of it."""
    rng = np.random.default_rng([seed, 5])
    # diagonal in the annulus, none within `gap` of the target except the planted one
    r = rng.uniform(1.0, 2.0, n)
    th = rng.uniform(0, 2 * np.pi, n)
    d = r * np.exp(1j * th)
    bad = np.abs(d - target) < gap
    while bad.any():
        d[bad] = rng.uniform(1.0, 2.0, bad.sum()) * np.exp(1j * rng.uniform(0, 2 * np.pi, bad.sum()))
        bad = np.abs(d - target) < gap
    p = n // 3
    d[p] = target
    rowptr = np.zeros(n + 1, dtype=np.int64)
    off_k = k - 1
    # off-diagonal columns uniform in (i, n): vectorised per row count min(off_k, n-1-i)
    cnt = np.minimum(off_k, n - 1 - np.arange(n))
    rowptr[1:] = np.cumsum(cnt + 1)
    nnz = int(rowptr[-1])
    colidx = np.empty(nnz, dtype=np.int64)
    values = np.empty(nnz, dtype=np.complex128)
    scale = 0.5 / max(off_k, 1)
    full = cnt == off_k
    idx_full = np.nonzero(full)[0]
    if idx_full.size:
        span = n - 1 - idx_full   # columns in (i, n) -> offsets in [0, span)
        u = rng.random((idx_full.size, off_k))
        # distinct offsets: sorted sample with arange trick on the per-row span
        r_ = np.floor(u * (span[:, None] - off_k + 1)).astype(np.int64)
        r_.sort(axis=1)
        r_ += np.arange(off_k)[None, :]
        oc = idx_full[:, None] + 1 + r_
        base = rowptr[idx_full]
        colidx[base[:, None] + np.arange(1, off_k + 1)[None, :]] = oc
        values[base[:, None] + np.arange(1, off_k + 1)[None, :]] = scale * (
            rng.uniform(-1, 1, (idx_full.size, off_k)) + 1j * rng.uniform(-1, 1, (idx_full.size, off_k)))
    for i in np.nonzero(~full)[0]:
        b = rowptr[i]
        c = int(cnt[i])
        colidx[b + 1: b + 1 + c] = np.arange(i + 1, i + 1 + c)
        values[b + 1: b + 1 + c] = scale * (rng.uniform(-1, 1, c) + 1j * rng.uniform(-1, 1, c))
    colidx[rowptr[:-1]] = np.arange(n)
    values[rowptr[:-1]] = d
    return rowptr.astype(np.int32), colidx.astype(np.int32), values, d


def general_complex(n: int, k: int, seed: int = 42, target=1.5 * np.exp(0.7j), gap: float = 0.05, sub: float = 0.3):
    """Non-triangular complex CSR with known eigenvalues (the general-sparse shifted-inverse case).

    triu_complex plus a subdiagonal entry A(i+1, i) = sub * e^{i phi} for every even i whose row i
    stores no (i, i+1): the matrix is block upper triangular with 2 x 2 diagonal blocks
    [[d_i, 0], [c, d_{i+1}]], so its eigenvalues are still the diagonal (planted target included),
    while no row/column permutation makes the pattern triangular for the solver's test.
    Returns (rowptr, colidx, values, diagonal)."""
    rp, ci, v, d = triu_complex(n, k, seed=seed, target=target, gap=gap)
    rp = rp.astype(np.int64)
    first_off = np.where(np.diff(rp) > 1, ci[np.minimum(rp[:-1] + 1, len(ci) - 1)], -1)
    i = np.arange(0, n - 1, 2)
    add = i[first_off[i] != i + 1]                  # (i, i+1) absent: the 2 x 2 block stays lower triangular
    phi = np.random.default_rng([seed, 6]).uniform(0, 2 * np.pi, add.size)
    rows = np.repeat(np.arange(n), np.diff(rp))
    rows = np.concatenate([rows, add + 1])
    cols = np.concatenate([ci.astype(np.int64), add])
    vals = np.concatenate([v, sub * np.exp(1j * phi)])
    order = np.lexsort((cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, rows + 1, 1)
    return np.cumsum(rowptr).astype(np.int32), cols.astype(np.int32), vals, d


def convdiff_complex(nx: int, seed: int = 2026, beta: float = 0.1, pert: float = 0.2, permute: bool = True):
    """General complex sparse matrix whose LU has real fill: a 2-D convection-diffusion 5-point
    stencil on an nx x nx grid (diagonal 4, neighbours -1 -/+ beta, -1 -/+ beta/2: nonsymmetric),
    every entry multiplied by 1 + pert * (u + i v), u, v ~ U(-1, 1), then a random symmetric
    permutation P A P^T (so neither the pattern nor its natural ordering is banded or triangular).
    n = nx^2, <= 5 entries per row; the spectrum lies around (0, 8) with clustered interior
    eigenvalues.  Returns (rowptr, colidx, values)."""
    rng = np.random.default_rng([seed, 9])
    n = nx * nx
    idx = np.arange(n, dtype=np.int64)
    ix, iy = idx % nx, idx // nx
    rows, cols = [idx], [idx]
    vals = [4.0 + pert * (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n))]
    for dx, dy, c in ((1, 0, -1 - beta), (-1, 0, -1 + beta), (0, 1, -1 - 0.5 * beta), (0, -1, -1 + 0.5 * beta)):
        m = (ix + dx >= 0) & (ix + dx < nx) & (iy + dy >= 0) & (iy + dy < nx)
        r = idx[m]
        rows.append(r)
        cols.append(r + dx + dy * nx)
        k = int(m.sum())
        vals.append(c * (1 + pert * (rng.uniform(-1, 1, k) + 1j * rng.uniform(-1, 1, k))))
    rows, cols, vals = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
    if permute:
        p = rng.permutation(n)            # new index of old row i: inv[i]; P A P^T
        inv = np.empty(n, np.int64)
        inv[p] = np.arange(n)
        rows, cols = inv[rows], inv[cols]
    order = np.lexsort((cols, rows))
    rows, cols, vals = rows[order], cols[order], vals[order]
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, rows + 1, 1)
    return np.cumsum(rowptr).astype(np.int32), cols.astype(np.int32), vals


def start_vector(n: int, dtype=np.float64, seed: int = 7, row0: int = 0) -> np.ndarray:
    """x0 of SURVEY §8d: U(-1, 1) per (re, im) component, seed 7 (normalised by the solver).
    Entries [row0, row0 + n) of the global start vector, drawn in the generators' fixed chunks, so
    a row block's slice is bitwise the slice of the N = 1 vector."""
    cx = np.issubdtype(np.dtype(dtype), np.complexfloating)
    x = np.empty(n, dtype=np.complex128 if cx else np.float64)
    for c, base, a, b in _chunks(row0, n):
        rng = np.random.default_rng([seed, c, 3])
        re = rng.uniform(-1.0, 1.0, CHUNK)
        if cx:
            x[a - row0:b - row0] = re[a - base:b - base] + 1j * rng.uniform(-1.0, 1.0, CHUNK)[a - base:b - base]
        else:
            x[a - row0:b - row0] = re[a - base:b - base]
    return x.astype(dtype)


def csr_bytes_per_iteration(n: int, nnz: int, scalar_bytes: int = 8) -> float:
    """Algorithmic HBM bytes of one fused power iteration."""
    return (scalar_bytes + 4.0) * nnz + 4.0 * (n + 1) + 2.0 * scalar_bytes * n
