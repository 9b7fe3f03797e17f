"""Torch-CPU fp32 restatement of the reference's train step (SURVEY §8(d)
``_cpu_ref``): the CPU baseline bench.py reports.

TEST INFRASTRUCTURE ONLY (see ae_oracle.py header): only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it.

The reference runs stock torch modules on its hot path, so its CPU cost is
that of these exact modules in the same order:

* FCLayer (layers/fc_layer.py:23-48): ``nn.Linear`` -> activation ->
  ``nn.BatchNorm1d`` (activation BEFORE BN, :38-45); the last layer of each
  FCModule is Linear only (modules/fc_module.py:34-51, model_builder.py:21-37);
* activation ``nn.LeakyReLU(0.2)`` (modules/activation.py:37-38);
* loss ``nn.MSELoss(reduction='sum')`` (modules/loss.py:31-32, model_builder.py:42);
* ``optim.Adam(model.parameters(), lr=1e-3)`` (novelty_detection.py:90);
* the step body of models/auto_encoder.py:57-77 (train, zero_grad, forward,
  loss, backward(retain_graph=True), optimizer.step, float(loss)).

The module tree mirrors the reference's so ``load_state_dict`` takes the same
60 keys; tests/test_oracle_golden.py pins it against the reference goldens.
"""
import torch
from torch import nn


class _FCLayer(nn.Module):
    """layers/fc_layer.py:23-48 (dropout 0)."""

    def __init__(self, fi, fo, act, bn):
        super().__init__()
        self.layer = nn.Linear(fi, fo)
        self.act = nn.LeakyReLU(0.2) if act else None
        self.bn = nn.BatchNorm1d(fo) if bn else None

    def forward(self, x):
        y = self.act(self.layer(x)) if self.act is not None else self.layer(x)
        if self.bn is not None:
            if y.dim() > 2:                       # layers/fc_layer.py:40-43
                shp = y.shape
                y = self.bn(y.reshape(-1, shp[-1])).reshape(shp)
            else:
                y = self.bn(y)
        return y


class _FCModule(nn.Module):
    def __init__(self, widths):
        super().__init__()
        n = len(widths) - 1
        self.net = nn.Sequential(*[_FCLayer(widths[i], widths[i + 1], i < n - 1, i < n - 1)
                                   for i in range(n)])

    def forward(self, x):
        return self.net(x)


class TorchRefAE(nn.Module):
    """models/auto_encoder.py:21-50 (encode -> view -> decode)."""

    def __init__(self, enc_widths, dec_widths):
        super().__init__()
        self.encoder = _FCModule(enc_widths)
        self.decoder = _FCModule(dec_widths)
        self.recon_loss = nn.MSELoss(reduction="sum")

    def forward(self, x):
        z = self.encoder(x).view(x.size(0), -1)
        return self.decoder(z).view(x.size(0), -1)


class TorchRefVIBAE(TorchRefAE):
    """The build-defined VIB-AE (SURVEY §8 a10/a10'): encoder emits mu|logvar
    (decorators/variational_info_bottleneck.py:34), z = eps*exp(logvar/2) + mu
    for k samples (:22-24,37), decoder on [k,B,btl]; loss = sum-MSE / k +
    beta * KL(N(mu, sigma) || N(0, 1))."""

    def __init__(self, enc_widths, dec_widths, k=1, beta_kl=1.0):
        super().__init__(enc_widths, dec_widths)
        self.k, self.beta_kl = k, beta_kl

    def vib_loss(self, x, eps=None):
        """eps: optional injected noise [k, B, btl] (tests); drawn otherwise."""
        out = self.encoder(x)
        mu, logvar = out.split(out.size(-1) // 2, dim=-1)
        sigma = (0.5 * logvar).exp()
        if eps is None:
            eps = torch.randn((self.k,) + mu.shape)
        z = eps * sigma + mu
        xh = self.decoder(z)
        recon = ((xh - x[None]) ** 2).sum() / self.k
        kl = -0.5 * (1 + logvar - mu * mu - logvar.exp()).sum()
        return recon + self.beta_kl * kl


def build(state_dict, enc_widths, dec_widths, vib=False, k=1, beta_kl=1.0):
    m = TorchRefVIBAE(enc_widths, dec_widths, k, beta_kl) if vib else TorchRefAE(enc_widths, dec_widths)
    m.load_state_dict({k: torch.as_tensor(v) for k, v in state_dict.items()})
    return m


def train_step(model, optimizer, x):
    """models/auto_encoder.py:57-77."""
    model.train()
    optimizer.zero_grad()
    if isinstance(model, TorchRefVIBAE):
        loss = model.vib_loss(x)
    else:
        loss = model.recon_loss(model(x), x)
    loss.backward(retain_graph=True)
    optimizer.step()
    return float(loss.detach())
