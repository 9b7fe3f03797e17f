"""GPU: the MFMA GEMM under split-K (in-launch combine of 2 or 4 K-slices).

Each layer-operator GEMM (forward with BN-statistic epilogue, bwd-data,
bwd-weight) is run with the split factor forced to 1, 2 and 4 through the
tuning knob and compared with a float64 torch reference of the same
contraction; the split result must be reproducible bit for bit run to run
(the slices combine in split order, whatever order they finish in), and every
launch must leave the split-K control words zero for the next one."""
import numpy as np
import pytest
import torch

from icra2021_multimodal_ad_amd import _native
from icra2021_multimodal_ad_amd._native import call, ptr, stream_ptr, pad, F32, BF16

pytestmark = pytest.mark.gpu

SHAPES = [(256, 300, 1000), (1024, 1658, 2048), (64, 100, 489), (512, 879, 1268)]


@pytest.fixture(scope="module")
def ws():
    w = _native.enable_gemm_workspace(torch.device("cuda", 0))
    yield w
    call("mmad_gemm_set_workspace", None, 0)


def _ctl_zero(ws):
    lib = _native.load()
    n = int(lib.mmad_gemm_ws_bytes())
    ctl = (8191 + 1) * 4                     # MMAD_SK_ERR_WORD + 1 words (csrc/mmad_gemm.h)
    slab = 832 * 128 * 128 * 4               # MMAD_SK_SLAB_TILES 128x128 fp32 tiles
    assert n == slab + ctl
    return int(ws[slab:n].view(torch.int32).abs().sum().item()) == 0


def _run(kind, dt, M, N, K, split):
    lib = _native.load()
    lib.mmad_tune_set(4, split)
    try:
        tdt = torch.bfloat16 if dt == BF16 else torch.float32
        g = torch.Generator(device="cuda").manual_seed(M * 7 + N * 3 + K)
        Mp, Np, Kp = pad(M), pad(N), pad(K)
        dev = torch.device("cuda", 0)
        s = stream_ptr()
        if kind == "fwd":
            x = torch.zeros(Mp, Kp, device=dev, dtype=tdt)
            x[:M, :K] = torch.randn(M, K, device=dev, generator=g).to(tdt)
            w = torch.zeros(Np, Kp, device=dev, dtype=tdt)
            w[:N, :K] = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(tdt)
            b = torch.zeros(Np, device=dev)
            b[:N] = torch.randn(N, device=dev, generator=g) * 0.1
            y = torch.empty(Mp, Np, device=dev, dtype=tdt)
            st = torch.empty(Mp // 32, 2, Np, device=dev)
            call("mmad_fc_fwd", dt, M, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 0, 0.0, None, None,
                 ptr(y), ptr(st), s)
            ref = x[:M, :K].double() @ w[:N, :K].double().t() + b[:N].double()
            return y[:M, :N].double(), ref
        if kind == "bwd_data":
            dz = torch.zeros(Mp, Np, device=dev, dtype=tdt)
            dz[:M, :N] = torch.randn(M, N, device=dev, generator=g).to(tdt)
            w = torch.zeros(Np, Kp, device=dev, dtype=tdt)
            w[:N, :K] = (torch.randn(N, K, device=dev, generator=g) * 0.05).to(tdt)
            dx = torch.empty(Mp, Kp, device=dev, dtype=tdt)
            call("mmad_fc_bwd_data", dt, M, N, K, Mp, Np, Kp, ptr(dz), ptr(w), ptr(dx), None, s)
            ref = dz[:M, :N].double() @ w[:N, :K].double()
            return dx[:M, :K].double(), ref
        # bwd_weight: dW[Np][Kp] = dz^T x, contraction over the batch M
        dz = torch.zeros(Mp, Np, device=dev, dtype=tdt)
        dz[:M, :N] = torch.randn(M, N, device=dev, generator=g).to(tdt)
        x = torch.zeros(Mp, Kp, device=dev, dtype=tdt)
        x[:M, :K] = torch.randn(M, K, device=dev, generator=g).to(tdt)
        dw = torch.empty(Np, Kp, device=dev)
        call("mmad_fc_bwd_weight", dt, Mp, Np, Kp, ptr(dz), ptr(x), ptr(dw), s)
        ref = dz[:M, :N].double().t() @ x[:M, :K].double()
        return dw[:N, :K].double(), ref
    finally:
        lib.mmad_tune_set(4, 0)


@pytest.mark.parametrize("dt", [F32, BF16])
@pytest.mark.parametrize("kind", ["fwd", "bwd_data", "bwd_weight"])
@pytest.mark.parametrize("shape", SHAPES)
def test_splitk_matches_reference_and_is_reproducible(ws, dt, kind, shape):
    M, N, K = shape
    outs = {}
    for split in (1, 2, 4):
        got, ref = _run(kind, dt, M, N, K, split)
        again, _ = _run(kind, dt, M, N, K, split)
        torch.cuda.synchronize()
        assert torch.equal(got, again), (kind, split)
        scale = ref.abs().max().item() + 1e-30
        err = (got - ref).abs().max().item() / scale
        # fp32 operands: fp32 accumulation error; bf16: output rounding to bf16
        tol = 2e-5 if dt == F32 else 1e-2 if kind != "bwd_weight" else 2e-5
        assert err < tol, (kind, split, err)
        outs[split] = got
        assert _ctl_zero(ws), (kind, split)
    # the split factors only reorder the fp32 accumulation
    for split in (2, 4):
        d = (outs[split] - outs[1]).abs().max().item() / (outs[1].abs().max().item() + 1e-30)
        assert d < (1e-5 if dt == F32 else 1e-2), (split, d)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_train_step_split_factors_agree(dtype):
    """The whole executor step with split-K forced off / 2 / 4: same loss and
    gradients to accumulation-order noise, identical across repeats."""
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data import synth_windows
    lib = _native.load()
    sd = init_state_dict(1728, 100, 5, seed=3)
    x = torch.from_numpy(synth_windows(1024, 1728, seed=4)).cuda()
    res = {}
    try:
        for split in (1, 2, 4, 2):
            lib.mmad_tune_set(4, split)
            cfg = types.SimpleNamespace(input_size=1728, btl_size=100, n_layers=5, gpu_id=0,
                                        dtype=dtype)
            m = get_model(cfg)
            m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
            loss = float(m._native.train_step(x))
            g = m._native.grads.clone()
            if split in res:
                assert loss == res[split][0] and torch.equal(g, res[split][1]), split
            res[split] = (loss, g)
    finally:
        lib.mmad_tune_set(4, 0)
    l1, g1 = res[1]
    for split in (2, 4):
        l, g = res[split]
        assert abs(l - l1) <= (1e-5 if dtype == "f32" else 1e-2) * abs(l1), (split, l, l1)
        cos = float(torch.nn.functional.cosine_similarity(g.double(), g1.double(), dim=0))
        # bf16: activations re-rounded per layer; the bf16-vs-fp32 bar of test_gpu_parity
        assert cos > (1 - 1e-6 if dtype == "f32" else 0.99), (split, cos)


@pytest.mark.parametrize("pair_rows", ["0", "1000"])
def test_shadow_pair_matches_single_shadow(monkeypatch, pair_rows):
    """bf16 fused steps with the ping-pong weight shadows (dW+Adam of a layer
    overlapping its bwd-data GEMM) give the same bits as the single-shadow
    schedule; the current shadow is always bf16(params).  pair_rows 0: every
    call ping-pongs; 1000: the executor alternates between the ping-pong
    schedule (1024-row calls) and the single-shadow one (512-row calls)."""
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.common_utils import init_state_dict
    from icra2021_multimodal_ad_amd.data import synth_windows
    sd = init_state_dict(1728, 100, 5, seed=5)
    xs = [torch.from_numpy(synth_windows(512 * (1 + i % 2), 1728, seed=10 + i)).cuda() for i in range(4)]
    res = {}
    for pair in ("1", "0"):
        cfg = types.SimpleNamespace(input_size=1728, btl_size=100, n_layers=5, gpu_id=0, dtype="bf16")
        with _native.tune(pair_rows=int(pair_rows), shadow_pair=pair == "1"):
            m = get_model(cfg)
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        assert m._native._pair == (pair == "1")
        losses = [float(m.train_step_async(x)) for x in xs]
        nat = m._native
        torch.cuda.synchronize()
        assert torch.equal(nat.shadow, nat.params[: nat.n_weight].bfloat16()), pair
        res[pair] = (losses, nat.params.clone())
    assert res["1"][0] == res["0"][0]
    assert torch.equal(res["1"][1], res["0"][1])


def test_splitk_timeout_is_reported_not_combined(ws):
    """A split-K combine that gives up waiting for a slice (forced here with
    the diagnostics knob) must not write a result built from stale slabs: the
    output tiles stay untouched and mmad_gemm_status reports MMAD_EHIP once."""
    lib = _native.load()
    M, N, K = 1024, 1658, 2048
    Mp, Np, Kp = pad(M), pad(N), pad(K)
    dev = torch.device("cuda", 0)
    x = torch.randn(Mp, Kp, device=dev).bfloat16()
    w = (torch.randn(Np, Kp, device=dev) * 0.05).bfloat16()
    b = torch.zeros(Np, device=dev)
    y = torch.full((Mp, Np), float("nan"), device=dev, dtype=torch.bfloat16)
    s = stream_ptr()
    assert lib.mmad_gemm_status(s) == 0
    lib.mmad_tune_set(4, 2)
    lib.mmad_tune_set(3, 4)
    try:
        call("mmad_fc_fwd", BF16, M, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 0, 0.0, None, None,
             ptr(y), None, s)
        rc = lib.mmad_gemm_status(s)
    finally:
        lib.mmad_tune_set(3, 0)
        lib.mmad_tune_set(4, 0)
    assert rc == _native.MMAD_EHIP
    assert b"timed out" in lib.mmad_last_error_string()
    assert torch.isnan(y.float()).all()          # no tile was combined from the slabs
    assert lib.mmad_gemm_status(s) == 0          # reported once, then cleared
    assert _ctl_zero(ws)
    # and the next (normal) launch is correct again
    call("mmad_fc_fwd", BF16, M, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 0, 0.0, None, None,
         ptr(y), None, s)
    ref = x[:M, :K].double() @ w[:N, :K].double().t()
    err = (y[:M, :N].double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2


@pytest.mark.parametrize("kind", ["fwd", "fwdns", "score", "mse"])
def test_persistent_grid_bit_identical(kind):
    """Knob 12 (persistent grid: one block per resident slot walks the tiles;
    1 and -1 alike) gives the ordinary grid's bits for the forward-type bf16 epilogues, with
    every large-row tile (256x128, 128x256, 256x256; tile 7 also issues the
    next tile's first K stages from its epilogue) forced, at a row count
    whose tiles exceed one resident round (16,384 rows: 512-1024 tiles on 256
    CUs); outputs, BN-statistic / score-row / loss partials compared."""
    lib = _native.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, K = 16384, 2048, 1658
    Mp, Np, Kp = pad(M), pad(N), pad(K)
    x = torch.zeros(Mp, Kp, device=dev, dtype=torch.bfloat16)
    x[:M, :K] = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = torch.zeros(Np, Kp, device=dev, dtype=torch.bfloat16)
    w[:N, :K] = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    b = torch.randn(Np, device=dev, generator=g) * 0.1
    ref = torch.randn(Mp, Np, device=dev, generator=g).bfloat16()
    tgt = torch.randn(M, N, device=dev, generator=g)
    s = stream_ptr()

    def run():
        y = torch.zeros(Mp, Np, device=dev, dtype=torch.bfloat16)
        part = torch.zeros(Mp // 32, 2, Np, device=dev)
        rows = torch.zeros(Np // 128, Mp, device=dev)
        if kind in ("fwd", "fwdns"):
            call("mmad_fc_fwd", BF16, M, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None, None,
                 ptr(y), ptr(part) if kind == "fwd" else None, s)
            return y, part
        if kind == "score":
            call("mmad_fc_fwd_score", BF16, M, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, None,
                 None, ptr(y), ptr(ref), ptr(rows), None, 0, s)
            return y, rows
        call("mmad_fc_fwd_mse", BF16, M, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), ptr(tgt), N, 2.0,
             ptr(y), ptr(part), s)
        return y, part
    try:
        for tile in (1, 2, 6, 7):
            lib.mmad_tune_set(0, tile)
            lib.mmad_tune_set(12, 0)
            a = run()
            for pk in (1, -1):                   # any nonzero value: persistent above one round
                lib.mmad_tune_set(12, pk)
                p = run()
                torch.cuda.synchronize()
                assert torch.equal(a[0], p[0]) and torch.equal(a[1], p[1]), (kind, tile, pk)
    finally:
        lib.mmad_tune_set(0, -1)
        lib.mmad_tune_set(12, 0)


@pytest.mark.parametrize("N", [2000, 1658])
@pytest.mark.parametrize("case", ["fwd_leaky_bn", "fwd_relu", "fwd_none", "score_ref_diff", "score_nodiff",
                                  "nap_colw", "fwd_stats_fallback", "fwd_sigmoid_fallback"])
def test_register_direct_tile_bit_identical(case, N):
    """Tiles 7, 8 and 9 (256x256 / 256x256 4-wave / 256x128 with the MFMA
    operands swapped, the epilogue stored from registers through
    v_permlane16_swap) against the row-quad tiles 6 / 1 / 2: bit-identical
    outputs, score row sums and diffs, on shapes with masked rows and columns
    (M = 4000 of 4096; N = 2000 of 2048, or 1658 of 1664, where only the
    256x128 / 128x... tiles fit and a forced 256x256 falls back to the tuned
    one).  The forward with
    BN-statistic partials and the sigmoid forward run CFG 6 in its place
    (same tile, same bits)."""
    lib = _native.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cuda").manual_seed(11)
    M, K = 4000, 1658
    Mp, Np, Kp = pad(M), pad(N), pad(K)
    x = torch.zeros(Mp, Kp, device=dev, dtype=torch.bfloat16)
    x[:M, :K] = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = torch.zeros(Np, Kp, device=dev, dtype=torch.bfloat16)
    w[:N, :K] = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    b = torch.randn(Np, device=dev, generator=g) * 0.1
    sc = 1.0 + 0.1 * torch.randn(Np, device=dev, generator=g)
    sh = 0.1 * torch.randn(Np, device=dev, generator=g)
    ref = torch.zeros(Mp, Np, device=dev, dtype=torch.bfloat16)
    ref[:M, :N] = torch.randn(M, N, device=dev, generator=g).bfloat16()
    colw = torch.zeros(Np, device=dev)
    colw[:N] = torch.rand(N, device=dev, generator=g) + 0.5
    s = stream_ptr()

    def run():
        y = torch.zeros(Mp, Np, device=dev, dtype=torch.bfloat16)
        rows = torch.zeros(Np // 128, Mp, device=dev)
        diff = torch.zeros(M, N, device=dev)
        part = torch.zeros(Mp // 32, 2, Np, device=dev)
        act = {"fwd_relu": 2, "fwd_none": 0, "fwd_sigmoid_fallback": 3}.get(case, 1)
        if case.startswith("fwd"):
            bn = case == "fwd_leaky_bn"
            call("mmad_fc_fwd", BF16, M, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), act, 0.2,
                 ptr(sc) if bn else None, ptr(sh) if bn else None, ptr(y),
                 ptr(part) if case == "fwd_stats_fallback" else None, s)
            return y, part
        if case == "nap_colw":
            score = torch.zeros(Mp, device=dev)
            call("mmad_nap_score", BF16, M, K, N, Mp, Kp, Np, ptr(x), ptr(w), ptr(b), ptr(colw),
                 ptr(rows), ptr(score), s)
            return rows, score
        call("mmad_fc_fwd_score", BF16, M, N, K, Mp, Np, Kp, ptr(x), ptr(w), ptr(b), 1, 0.2, ptr(sc),
             ptr(sh), ptr(y), ptr(ref), ptr(rows),
             ptr(diff) if case == "score_ref_diff" else None, N, s)
        return y, rows, diff
    outs = {}
    try:
        for tile in (6, 7, 8, 1, 2, 9):
            lib.mmad_tune_set(0, tile)
            outs[tile] = run()
        torch.cuda.synchronize()
    finally:
        lib.mmad_tune_set(0, -1)
    assert float(outs[6][0].float().abs().sum()) > 0
    for tile in (7, 8, 1, 2, 9):
        for a, b2 in zip(outs[6], outs[tile]):
            assert torch.equal(a, b2), (case, tile)


@pytest.mark.parametrize("blocks", [256, 512])
def test_f32_dw_split_rule_fused_step(blocks):
    """Knob 32 (the exact-fp32 path's dW split-K rule from 2048 rows) at the
    C3 shape through the fused step (dW with the Adam epilogue run by the
    last arriving slice): every split dW layer's slices combined in split
    order -- repeat runs identical bit for bit -- and the step equal to the
    unsplit one to fp32 accumulation order after the first step: loss within
    1e-6, Adam moments within 1e-5 of their scale, parameters within 1e-6 but for
    sign-of-zero gradient entries (<= 1e-4 of them); forward-type GEMMs and
    batches below 2048 rows never split."""
    import types
    from icra2021_multimodal_ad_amd.model_builder import get_model
    from icra2021_multimodal_ad_amd.data import synth_windows
    lib = _native.load()
    with _native.tune(splitk_dw_f32_blocks=0):
        assert lib.mmad_gemm_splitk_for(512, 128, 4096, F32, 3) == 1      # knob off: no split
    xs = [torch.from_numpy(synth_windows(4096, 2048, seed=30 + i)).cuda() for i in range(2)]
    eps = torch.randn(1, 4096, 100, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    res = []
    for knob in (0, blocks, blocks):
        with _native.tune(splitk_dw_f32_blocks=knob):
            if knob:
                assert lib.mmad_gemm_splitk_for(512, 128, 4096, F32, 3) > 1   # L5's dW: [512 x 128], K 4096
                assert lib.mmad_gemm_splitk_for(512, 128, 1024, F32, 3) == 1  # below 2048 rows
                assert lib.mmad_gemm_splitk_for(4096, 128, 512, F32, 0) == 1  # forward
            cfg = types.SimpleNamespace(input_size=2048, btl_size=100, n_layers=5, gpu_id=0, dtype="f32",
                                        models="vib_ae", vib_k=1, beta_kl=1.0)
            torch.manual_seed(33)
            m = get_model(cfg)
            nat = m._native
            run = []
            for x in xs:
                loss = float(nat.train_step_fused(x, k=1, eps=eps, beta_kl=1.0))
                torch.cuda.synchronize()
                run.append((loss, nat.params.clone(), nat.exp_avg.clone(), nat.exp_avg_sq.clone()))
            nat.check_status()
            res.append(run)
    # the split schedule is reproducible bit for bit over both steps
    for (la, pa, ma, va), (lb, pb, mb, vb) in zip(res[1], res[2]):
        assert la == lb and torch.equal(pa, pb) and torch.equal(ma, mb) and torch.equal(va, vb)
    # against the unsplit step: the first step (the second one's inputs
    # already differ by the first one's sign-of-zero entries, below)
    (l0, p0, m0, v0), (l1, p1, m1, v1) = res[0][0], res[1][0]
    assert abs(l0 - l1) <= 1e-6 * abs(l0), (l0, l1)
    # Adam's moments carry the gradient: a dW entry is a 4096-row sum whose
    # terms may cancel, so another fp32 order moves it by ~2^-24 of the terms'
    # magnitude, not of its own (measured 1.7e-6 of max|m|); the parity bar
    # for fp32 gradients is 1e-4 of their max (test_gpu_parity)
    for a, b in ((m0, m1), (v0, v1)):
        assert float((a - b).abs().max()) <= 1e-5 * float(a.abs().max())
    # parameters: Adam's first steps move each weight by ~lr * sign(g), so an
    # entry whose gradient is zero to rounding may step the other way; all but
    # such entries agree to fp32 accumulation order
    far = (p0 - p1).abs() > 1e-6 * float(p0.abs().max())
    assert float(far.double().mean()) <= 1e-4, int(far.sum())
