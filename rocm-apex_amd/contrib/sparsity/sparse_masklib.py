"""N:M structured-sparsity masks (reference apex/contrib/sparsity/sparse_masklib.py:9-184).

Pattern names follow the reference: ``m4n2_1d`` (in every group of 4 consecutive input
elements keep the 2 largest |w|), ``m4n2_2d_greedy`` / ``m4n2_2d_best`` (4x4 blocks with 2 kept
per row AND per column, for weights used transposed in the backward pass).  All patterns are
computed with batched tensor ops on the weight's own device (one pass per layer, no python
loops over groups): 1-D and 2-D "best" score every candidate pattern with one matmul.
"""
import itertools
import sys

import torch

_pattern_cache = {}


def valid_1d_patterns(m, n, device):
    key = ("1d", m, n, str(device))
    if key not in _pattern_cache:
        pats = [[1.0 if i in keep else 0.0 for i in range(m)] for keep in itertools.combinations(range(m), n)]
        _pattern_cache[key] = torch.tensor(pats, device=device)
    return _pattern_cache[key]


def valid_2d_patterns(m, n, device):
    """All m x m 0/1 blocks with exactly n ones in every row and every column."""
    key = ("2d", m, n, str(device))
    if key not in _pattern_cache:
        rows = [tuple(1.0 if i in keep else 0.0 for i in range(m)) for keep in itertools.combinations(range(m), n)]
        pats = []
        for combo in itertools.product(rows, repeat=m):
            if all(sum(r[c] for r in combo) == n for c in range(m)):
                pats.append(combo)
        _pattern_cache[key] = torch.tensor(pats, device=device)  # [P, m, m]
    return _pattern_cache[key]


def _groups_1d(mat, m):
    """[R, C] -> [R * ceil(C/m), m] (zero padded), plus the padded width."""
    r, c = mat.shape
    pad = (-c) % m
    if pad:
        mat = torch.nn.functional.pad(mat, (0, pad))
    return mat.reshape(-1, m), c + pad


def mn_1d_best(matrix, m, n):
    groups, width = _groups_1d(matrix.abs(), m)
    pats = valid_1d_patterns(m, n, matrix.device)
    choice = torch.argmax(groups @ pats.t(), dim=1)
    mask = pats[choice].reshape(matrix.size(0), width)[:, :matrix.size(1)]
    return mask.contiguous()


def m4n2_1d(mat, density):
    return mn_1d_best(mat, 4, 2)


def _blocks_2d(mat, m):
    r, c = mat.shape
    pr, pc = (-r) % m, (-c) % m
    if pr or pc:
        mat = torch.nn.functional.pad(mat, (0, pc, 0, pr))
    R, C = mat.shape
    blocks = mat.reshape(R // m, m, C // m, m).permute(0, 2, 1, 3).reshape(-1, m, m)
    return blocks, R, C


def _unblock_2d(blocks, R, C, m, r, c):
    return blocks.reshape(R // m, C // m, m, m).permute(0, 2, 1, 3).reshape(R, C)[:r, :c].contiguous()


def mn_2d_best(matrix, m, n):
    blocks, R, C = _blocks_2d(matrix.abs(), m)
    pats = valid_2d_patterns(m, n, matrix.device)  # [P, m, m]
    score = blocks.reshape(-1, m * m) @ pats.reshape(-1, m * m).t()
    choice = torch.argmax(score, dim=1)
    return _unblock_2d(pats[choice], R, C, m, *matrix.shape)


def m4n2_2d_best(mat, density):
    return mn_2d_best(mat, 4, 2)


def mn_2d_greedy(matrix, m, n):
    """Per block: visit entries by decreasing |w| and keep one while its row and column have
    fewer than n kept.  Vectorised over blocks (m*m sequential steps)."""
    blocks, R, C = _blocks_2d(matrix.abs(), m)
    nb = blocks.size(0)
    order = torch.argsort(blocks.reshape(nb, -1), dim=1, descending=True)
    mask = torch.zeros(nb, m * m, device=matrix.device)
    row_cnt = torch.zeros(nb, m, device=matrix.device)
    col_cnt = torch.zeros(nb, m, device=matrix.device)
    ar = torch.arange(nb, device=matrix.device)
    for step in range(m * m):
        idx = order[:, step]
        r, c = idx // m, idx % m
        ok = (row_cnt[ar, r] < n) & (col_cnt[ar, c] < n)
        mask[ar, idx] = torch.where(ok, torch.ones_like(mask[ar, idx]), mask[ar, idx])
        row_cnt[ar, r] += ok.float()
        col_cnt[ar, c] += ok.float()
    return _unblock_2d(mask.reshape(nb, m, m), R, C, m, *matrix.shape)


def m4n2_2d_greedy(mat, density):
    return mn_2d_greedy(mat, 4, 2)


def create_mask(tensor, pattern="m4n2_1d", density=0.5):
    """Mask of ``tensor``'s shape/dtype.  Groups run along the input dimension: dim 1 of a
    Linear weight [out, in]; for a conv weight [K, C, R, S] along C (as [R*S*K, C])."""
    func = pattern if callable(pattern) else getattr(sys.modules[__name__], pattern)
    shape = tensor.shape
    t = tensor.detach().float().contiguous()
    if t.dim() == 1:
        mask = func(t.view(1, -1), density)
    elif t.dim() == 2:
        mask = func(t, density)
    elif t.dim() == 3:
        mask = func(t.view(shape[0] * shape[1], shape[2]), density)
    elif t.dim() == 4:
        k, c, r, s = shape
        mask = func(t.permute(2, 3, 0, 1).reshape(r * s * k, c), density)
        mask = mask.view(r, s, k, c).permute(2, 3, 0, 1)
    else:
        raise ValueError("create_mask: unsupported tensor rank {}".format(t.dim()))
    return mask.reshape(shape).to(tensor.dtype)
