"""CPU oracle for the HSR_Net multimodal fusion producer.

TEST INFRASTRUCTURE ONLY (same contract as ``oracle/ae_oracle.py``): only
``tests/`` and the CPU-baseline legs of the benches may import it; the product
path (``icra2021_multimodal_ad_amd.hsr_net``) never imports or falls back to it.

A plain-numpy fp32 restatement of ``HSR_Net.forward`` (utils/data_loaders.py:
179-229) for the modalities the reference feeds it (r, d, t, m; the 1-D LiDAR
branch is never called by the reference: l is None at :401 and :405-424).
Pinned by ``tests/golden/hsr.npz`` (``tests/golden/gen_hsr_golden.py`` runs
the reference itself); ``tests/test_oracle_golden.py`` checks the pin.

Weights: a dict of the reference state_dict names (``conv1r.weight`` ...).
"""
import numpy as np

F32 = np.float32


def conv2d(x, w, b, stride, pad):
    """torch.nn.Conv2d on [n, ci, h, w] (cross-correlation, zero padding)."""
    n, ci, h, wd = x.shape
    co, _, kh, kw = w.shape
    if pad:
        x = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    ho = (h + 2 * pad - kh) // stride + 1
    wo = (wd + 2 * pad - kw) // stride + 1
    out = np.zeros((n, co, ho, wo), F32)
    for ky in range(kh):
        for kx in range(kw):
            patch = x[:, :, ky:ky + stride * ho:stride, kx:kx + stride * wo:stride]  # n ci ho wo
            out += np.einsum("nchw,oc->nohw", patch, w[:, :, ky, kx]).astype(F32)
    return out + b[None, :, None, None].astype(F32)


def _conv1d(x, w, b, stride, pad):
    """torch.nn.Conv1d on [n, ci, L] (zero padding)."""
    n, ci, L = x.shape
    co, _, k = w.shape
    x = np.pad(x, ((0, 0), (0, 0), (pad, pad)))
    lo = (L + 2 * pad - k) // stride + 1
    out = np.zeros((n, co, lo), F32)
    for t in range(k):
        patch = x[:, :, t:t + stride * lo:stride]
        out += np.einsum("ncl,oc->nol", patch, w[:, :, t]).astype(F32)
    return out + b[None, :, None].astype(F32)


def relu(x):
    return np.maximum(x, 0).astype(F32)


def rgb_branch(W, r):
    """:186-191 -- r [n,3,32,32] -> [n,16,8,8]."""
    x = relu(conv2d(r, W["conv1r.weight"], W["conv1r.bias"], 2, 0))
    x = relu(conv2d(x, W["conv2r.weight"], W["conv2r.bias"], 1, 1))
    return relu(conv2d(x, W["conv3r.weight"], W["conv3r.bias"], 2, 0))


def depth_branch(W, d):
    """:193-198 -- d [n,1,32,32] -> [n,8,8,8]."""
    x = relu(conv2d(d, W["conv1d.weight"], W["conv1d.bias"], 2, 0))
    x = relu(conv2d(x, W["conv2d.weight"], W["conv2d.bias"], 1, 1))
    return relu(conv2d(x, W["conv3d.weight"], W["conv3d.bias"], 2, 0))


def ft_branch(t):
    """:211-213 -- t [n] -> [n,1,8,8] (scalar broadcast)."""
    return np.broadcast_to(t.reshape(-1, 1, 1, 1), (t.shape[0], 1, 8, 8)).astype(F32)


def mic_branch(W, m):
    """:217-220 -- m [n,13] -> [n,2,8,8]: the LiDAR convs conv1l/conv2l (the
    reference reuses them for the mic), view(-1,2,8,1), repeat x8 along w."""
    x = relu(_conv1d(m[:, None, :], W["conv1l.weight"], W["conv1l.bias"], 9, 9))
    x = relu(_conv1d(x, W["conv2l.weight"], W["conv2l.bias"], 2, 0))      # [n,16,1]
    return np.repeat(x.reshape(-1, 2, 8, 1), 8, axis=3)


def hsr_forward(W, r=None, d=None, t=None, m=None, unimodal=False):
    """HSR_Net.forward(r, d, None, t, m) (:179-229) over a batch, flattened to
    rows: All -> [n,1728] = cat(rr, dd, tt, mm) channel-major (:223-224);
    unimodal -> the last given modality's block (:190-221 overwrite order)."""
    blocks = []
    if r is not None:
        blocks.append(rgb_branch(W, np.asarray(r, F32).reshape(-1, 3, 32, 32)))
    if d is not None:
        blocks.append(depth_branch(W, np.asarray(d, F32).reshape(-1, 1, 32, 32)))
    if t is not None:
        blocks.append(ft_branch(np.asarray(t, F32).reshape(-1)))
    if m is not None:
        blocks.append(mic_branch(W, np.asarray(m, F32).reshape(-1, 13)))
    if unimodal:
        out = blocks[-1]
    else:
        if r is None or d is None or t is None or m is None:
            raise NameError("HSR_Net: the concatenation needs r, d, t and m (data_loaders.py:224)")
        out = np.concatenate(blocks, axis=1)
    return out.reshape(out.shape[0], -1)
