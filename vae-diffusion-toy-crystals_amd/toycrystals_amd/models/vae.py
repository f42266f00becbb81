"""MI355X-native drop-in for toycrystals.models.vae (CondVAE / VAE).

Mirrors /root/reference/src/toycrystals/models/vae.py:8-134 (same names, constructor
signatures, attributes and state_dict keys; seeded init identical).  encode/decode run in
libtcx: the four 4x4/s2 zero-padded encoder convs and the FCs as fp32-MFMA implicit GEMMs
with fused ReLU, the decoder's ConvTranspose2d(4, s2, p1) as four sub-pixel phase GEMMs with
fused ReLU / sigmoid.  Activations are NHWC inside; the flatten/view of the 256x4x4 map is
folded into a column/row permutation of enc_fc / dec_fc at pack time.
The reparameterisation noise and the training-time condition dropout draw from torch's RNG
in the reference's order (vae.py:57-60, 65-67); the one-hot/concat condition vector, the
keep mask and the reparameterisation run in libtcx kernels (tcx_vae_yvec, tcx_reparam).

Training: with autograd on (grad enabled and parameters requiring grad) the same forward runs
as a chain of libtcx autograd Functions (functional.py): Conv2d(4,2,1)+ReLU encoder, the NCHW
flatten as an explicit [16][256] -> [256][16] transpose, FCs on the fp32-MFMA GEMM,
ConvTranspose2d phases, Sigmoid; `kl_stats` (train_vae.py:17-36) is functional.kl_stats.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import functional as TF
from .._lib import check, lib, ptr, require_gpu_tensor, stream_ptr


def _round_up(v: int, a: int) -> int:
    return (v + a - 1) // a * a


class _VAEPack:
    def __init__(self, m: "_VAEBase", device: torch.device) -> None:
        L = lib()
        st = stream_ptr(device)
        self.keep = []

        def dev(t):
            t = t.detach().to(device=device, dtype=torch.float32).contiguous()
            self.keep.append(t)
            return t

        def pack(w4: torch.Tensor):  # [Cout][Cin][k][k]
            w4 = dev(w4)
            cout, cin, ks, _ = w4.shape
            kpad, cpad = _round_up(ks * ks * cin, 32), _round_up(cout, 32)
            wpk = torch.empty((cpad, kpad), device=device, dtype=torch.float32)
            check(L.tcx_pack_conv_weight(ptr(w4), ptr(wpk), cout, cin, ks, cpad, kpad, st), "pack")
            self.keep.append(wpk)
            return (wpk, cout, cpad, kpad, cin)

        self.enc = [(pack(m.enc[i].weight), dev(m.enc[i].bias)) for i in (0, 2, 4, 6)]
        # enc_fc: reference flattens NCHW [256,4,4] (c*16 + y*4 + x); we flatten NHWC ((y*4+x)*256 + c)
        w = m.enc_fc.weight.detach()
        n_img = 256 * 16
        w_img = w[:, :n_img].reshape(w.shape[0], 256, 16).transpose(1, 2).reshape(w.shape[0], n_img)
        w_fc = torch.cat([w_img, w[:, n_img:]], dim=1)
        self.enc_fc = (pack(w_fc[:, :, None, None]), dev(m.enc_fc.bias))
        # mu and logvar as one 256 -> 2z GEMM
        self.heads = (pack(torch.cat([m.mu.weight, m.logvar.weight], 0)[:, :, None, None]),
                      dev(torch.cat([m.mu.bias, m.logvar.bias], 0)))
        # dec_fc rows permuted so its output is the NHWC [4,4,256] map
        wd, bd = m.dec_fc.weight.detach(), m.dec_fc.bias.detach()
        perm = torch.arange(n_img).reshape(256, 16).t().reshape(-1)  # new row (yx*256 + c) <- old (c*16 + yx)
        self.dec_fc = (pack(wd[perm][:, :, None, None]), dev(bd[perm]))
        self.dec = []
        for i in (0, 2, 4, 6):
            ct = m.dec[i]
            wT = dev(ct.weight)  # [Cin][Cout][4][4]
            cin, cout = wT.shape[0], wT.shape[1]
            kpad, cpad = _round_up(4 * cin, 32), _round_up(cout, 32)
            wpk = torch.empty((4, cpad, kpad), device=device, dtype=torch.float32)
            check(L.tcx_pack_convT_weight(ptr(wT), ptr(wpk), cin, cout, cpad, kpad, st), "packT")
            self.keep.append(wpk)
            self.dec.append((wpk, cin, cout, cpad, kpad, dev(ct.bias)))


def _linear(x1, x2, packed, bias, act, resid=None):
    (wpk, n, npad, kpad, k) = packed
    M = x1.shape[0]
    K1 = x1.shape[1]
    K2 = x2.shape[1] if x2 is not None else 0
    assert K1 + K2 == k
    y = torch.empty((M, n), device=x1.device, dtype=torch.float32)
    nb = int(lib().tcx_linear_workspace(M, n, K1, K2))
    ws = TF._ws(x1.device, nb) if nb else None
    check(lib().tcx_linear_ws(ptr(x1), K1, ptr(x2), K2, ptr(wpk), ptr(bias), ptr(resid), ptr(y), M, n, npad, kpad,
                              act, ptr(ws), nb, stream_ptr(x1.device)), "tcx_linear")
    return y


class _VAEBase(nn.Module):
    def _tcx(self, device):
        if device.type != "cuda":
            raise RuntimeError("the VAE runs on the MI355X only: move the model and inputs to 'cuda'")
        key = (device,) + tuple((p.data_ptr(), p._version) for p in self.parameters())
        if getattr(self, "_pk_key", None) != key:
            with torch.no_grad():
                self._pk = _VAEPack(self, device)
            self._pk_key = key
        return self._pk

    def _encode_img(self, x: torch.Tensor) -> torch.Tensor:
        """4 x [Conv4x4 s2 p1 (zero) + ReLU]: [B,1,64,64] -> NHWC [B,4,4,256] flattened [B,4096]."""
        require_gpu_tensor(x, "x")
        pk = self._tcx(x.device)
        st = stream_ptr(x.device)
        h = x.float().contiguous()
        B, _, H, W = h.shape
        for (wpk, cout, cpad, kpad, cin), b in pk.enc:
            Ho, Wo = H // 2, W // 2
            y = torch.empty((B, Ho, Wo, cout), device=x.device, dtype=torch.float32)
            check(lib().tcx_conv2d(ptr(h), None, B, 0, H, W, cin, 0, ptr(wpk), ptr(b), None, None, ptr(y), cout, cpad,
                                   kpad, 4, 2, 1, 0, 0, 1, None, None, None, None, None, st), "enc conv")
            h, H, W = y, Ho, Wo
        return h.reshape(B, -1)

    def _decode_map(self, h: torch.Tensor) -> torch.Tensor:
        """[B, 4*4*256] NHWC map -> 4 x ConvT(4, s2, p1) (+ReLU, last +sigmoid) -> [B,1,64,64]."""
        pk = self._pk
        st = stream_ptr(h.device)
        B = h.shape[0]
        H = W = 4
        for j, (wpk, cin, cout, cpad, kpad, b) in enumerate(pk.dec):
            y = torch.empty((B, 2 * H, 2 * W, cout), device=h.device, dtype=torch.float32)
            act = 2 if j == 3 else 1
            check(lib().tcx_convT2x(ptr(h), B, H, W, cin, ptr(wpk), ptr(b), ptr(y), cout, cpad, kpad, act, st),
                  "dec convT")
            h, H, W = y, 2 * H, 2 * W
        return h.reshape(B, 1, H, W)  # C == 1: NHWC == NCHW

    def _grad_mode(self) -> bool:
        return torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())

    def reparameterise(self, mu: torch.Tensor, logvar: torch.Tensor, eps: torch.Tensor = None) -> torch.Tensor:
        """mu + exp(0.5 logvar) * eps, eps = randn_like(std) (vae.py:57-60)."""
        mu, logvar = mu.float().contiguous(), logvar.float().contiguous()
        if eps is None:
            eps = torch.randn_like(mu)
        eps = eps.to(device=mu.device, dtype=torch.float32).contiguous()
        if torch.is_grad_enabled() and (mu.requires_grad or logvar.requires_grad):
            return TF.ReparamFn.apply(mu, logvar, eps)
        z = torch.empty_like(mu)
        check(lib().tcx_reparam(ptr(mu), ptr(logvar), ptr(eps), mu.numel(), ptr(z), stream_ptr(mu.device)),
              "tcx_reparam")
        return z

    # ---------------------------------------------------------------- training path (autograd)
    def _enc_train(self, x: torch.Tensor, y: torch.Tensor = None):
        require_gpu_tensor(x, "x")
        B = x.shape[0]
        h = x.float().contiguous().view(B, x.shape[2], x.shape[3], 1)
        for i in (0, 2, 4, 6):
            h = TF.act(TF.conv2d(h, None, self.enc[i]), TF.ACT_RELU)
        _, Hh, Wh, Ch = h.shape
        hf = TF.TransposeBHCFn.apply(h.view(B, Hh * Wh, Ch)).view(B, Ch * Hh * Wh)  # h.flatten(1) of NCHW
        if y is not None:
            hf = TF.cat_cols(hf, y)
        h = TF.act(TF.linear(hf, self.enc_fc), TF.ACT_RELU)
        return TF.linear(h, self.mu), TF.linear(h, self.logvar)

    def _dec_train(self, zc: torch.Tensor):
        B = zc.shape[0]
        hd = TF.linear(zc, self.dec_fc)  # [B, 256*4*4] in the reference's .view(-1, 256, 4, 4) order
        hd = TF.TransposeBHCFn.apply(hd.view(B, 256, 16)).view(B, 4, 4, 256)
        for j, i in enumerate((0, 2, 4, 6)):
            ct = self.dec[i]
            hd = TF.act(TF.ConvTranspose2xFn.apply(hd, ct.weight, ct.bias), TF.ACT_SIGMOID if j == 3 else TF.ACT_RELU)
        return hd.view(B, 1, hd.shape[1], hd.shape[2])


class CondVAE(_VAEBase):
    def __init__(self, z_dim: int = 16, n_types: int = 4, y_cont_dim: int = 4, cond_drop: float = 0.1) -> None:
        super().__init__()
        self.z_dim = z_dim
        self.n_types = n_types
        self.y_cont_dim = y_cont_dim
        self.y_dim = n_types + y_cont_dim
        self.cond_drop = float(cond_drop)
        self.enc = nn.Sequential(
            nn.Conv2d(1, 32, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(32, 64, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(64, 128, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(128, 256, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
        )
        self.enc_fc = nn.Linear(256 * 4 * 4 + self.y_dim, 256)
        self.mu = nn.Linear(256, z_dim)
        self.logvar = nn.Linear(256, z_dim)
        self.dec_fc = nn.Linear(z_dim + self.y_dim, 256 * 4 * 4)
        self.dec = nn.Sequential(
            nn.ConvTranspose2d(256, 128, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.ConvTranspose2d(128, 64, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.ConvTranspose2d(64, 32, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.ConvTranspose2d(32, 1, kernel_size=4, stride=2, padding=1), nn.Sigmoid(),
        )

    def _y_vec(self, y_cat: torch.Tensor, y_cont: torch.Tensor, keep_u: torch.Tensor = None) -> torch.Tensor:
        """[one_hot(y_cat) | y_cont] (vae.py:45-48), optionally times the keep mask (vae.py:65-67)."""
        y_cat = y_cat.to(torch.int64).contiguous()
        y_cont = y_cont.to(device=y_cat.device, dtype=torch.float32).contiguous()
        B = y_cat.shape[0]
        out = torch.empty((B, self.y_dim), device=y_cat.device, dtype=torch.float32)
        check(lib().tcx_vae_yvec(ptr(y_cat), ptr(y_cont), ptr(keep_u), float(self.cond_drop), B, self.n_types,
                                 self.y_cont_dim, ptr(out), stream_ptr(y_cat.device)), "tcx_vae_yvec")
        return out

    def _keep_u(self, B: int, device, keep_u=None):
        if self.training and self.cond_drop > 0.0:
            if keep_u is None:
                keep_u = torch.rand((B, 1), device=device)
            return keep_u.to(device=device, dtype=torch.float32).contiguous()
        return None

    def encode(self, x, y_cat, y_cont):
        if self._grad_mode():
            return self._enc_train(x, self._y_vec(y_cat, y_cont))
        with torch.no_grad():
            h = self._encode_img(x)
            y = self._y_vec(y_cat, y_cont)
            h = _linear(h, y, self._pk.enc_fc[0], self._pk.enc_fc[1], act=1)
            ml = _linear(h, None, self._pk.heads[0], self._pk.heads[1], act=0)
            return ml[:, :self.z_dim].contiguous(), ml[:, self.z_dim:].contiguous()

    def decode(self, z, y_cat, y_cont, *, keep_u: torch.Tensor = None):
        require_gpu_tensor(z, "z")
        y = self._y_vec(y_cat, y_cont, self._keep_u(z.shape[0], z.device, keep_u))
        if self._grad_mode():
            return self._dec_train(TF.cat_cols(z.float(), y))
        with torch.no_grad():
            pk = self._tcx(z.device)
            h = _linear(z.float().contiguous(), y, pk.dec_fc[0], pk.dec_fc[1], act=0)
            return self._decode_map(h)

    def forward(self, x, y_cat, y_cont, *, draws=None):
        """x_hat, mu, logvar (vae.py:70-78).  draws = (reparam eps [B,z], keep_u [B,1]) injects the
        reference's two RNG draws (randn_like then rand) for parity runs."""
        eps, keep_u = draws if draws is not None else (None, None)
        mu, logvar = self.encode(x, y_cat, y_cont)
        z = self.reparameterise(mu, logvar, eps)
        return self.decode(z, y_cat, y_cont, keep_u=keep_u), mu, logvar


class VAE(_VAEBase):
    """Unconditional VAE baseline (vae.py:81-134)."""

    def __init__(self, z_dim: int = 16) -> None:
        super().__init__()
        self.z_dim = z_dim
        self.enc = nn.Sequential(
            nn.Conv2d(1, 32, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(32, 64, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(64, 128, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.Conv2d(128, 256, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
        )
        self.enc_fc = nn.Linear(256 * 4 * 4, 256)
        self.mu = nn.Linear(256, z_dim)
        self.logvar = nn.Linear(256, z_dim)
        self.dec_fc = nn.Linear(z_dim, 256 * 4 * 4)
        self.dec = nn.Sequential(
            nn.ConvTranspose2d(256, 128, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.ConvTranspose2d(128, 64, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.ConvTranspose2d(64, 32, kernel_size=4, stride=2, padding=1), nn.ReLU(inplace=True),
            nn.ConvTranspose2d(32, 1, kernel_size=4, stride=2, padding=1), nn.Sigmoid(),
        )

    def encode(self, x):
        if self._grad_mode():
            return self._enc_train(x)
        with torch.no_grad():
            h = self._encode_img(x)
            h = _linear(h, None, self._pk.enc_fc[0], self._pk.enc_fc[1], act=1)
            ml = _linear(h, None, self._pk.heads[0], self._pk.heads[1], act=0)
            return ml[:, :self.z_dim].contiguous(), ml[:, self.z_dim:].contiguous()

    def decode(self, z):
        require_gpu_tensor(z, "z")
        if self._grad_mode():
            return self._dec_train(z.float())
        with torch.no_grad():
            pk = self._tcx(z.device)
            h = _linear(z.float().contiguous(), None, pk.dec_fc[0], pk.dec_fc[1], act=0)
            return self._decode_map(h)

    def forward(self, x, *, draws=None):
        eps = draws[0] if draws is not None else None
        mu, logvar = self.encode(x)
        z = self.reparameterise(mu, logvar, eps)
        return self.decode(z), mu, logvar
