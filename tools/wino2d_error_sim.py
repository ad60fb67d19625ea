"""CPU simulation of the f16x3 error of the 3x3 conv forms, against a float64 conv on the same inputs:
direct (9 taps), Winograd F(2,3) along x (the shipped wc_conv3x3_wino_f16x3) and 2D F(2x2,3x3) (the
candidate).  Operands as the kernels form them: transformed input in fp32, times a power of
two, split into two round-to-nearest fp16 pieces; filter transform in float64, per-output-channel power
of two, one rounding to fp32, two fp16 pieces; products h*h + h*l + l*h exact, fp32 accumulation over
16-channel chunks.  Usage: python tools/wino2d_error_sim.py [--c 128] [--n 64] [--hw 32]"""
import argparse

import torch

BT = torch.tensor([[1., 0., -1., 0.], [0., 1., 1., 0.], [0., -1., 1., 0.], [0., 1., 0., -1.]], dtype=torch.float64)
G = torch.tensor([[1., 0., 0.], [.5, .5, .5], [.5, -.5, .5], [0., 0., 1.]], dtype=torch.float64)
AT = torch.tensor([[1., 1., 1., 0.], [0., 1., -1., -1.]], dtype=torch.float64)


def split2(v32):
    """v (fp32) -> (h, l) fp16 pieces as fp32 values: h = fp16(v), l = fp16(v - h)."""
    h = v32.half().float()
    return h, (v32 - h).half().float()


def pow2_scale(amax, target=2.0**14):
    e = torch.floor(torch.log2(target / amax.clamp_min(1e-300)))
    return torch.pow(2.0, e)


def f16x3_gemm(a, b):
    """a [M][K], b [K][N] (float64 values, already power-of-two scaled): fp32 rounding, split, three
    exact products, fp32 accumulation in 16-wide K chunks (the MFMA's K-step)."""
    ah, al = split2(a.float())
    bh, bl = split2(b.float())
    out = torch.zeros((a.shape[0], b.shape[1]), dtype=torch.float32)
    for k0 in range(0, a.shape[1], 16):
        s = slice(k0, k0 + 16)
        part = (ah[:, s].double() @ bh[s].double() + ah[:, s].double() @ bl[s].double()
                + al[:, s].double() @ bh[s].double())  # exact products, summed (the MFMA sums them in fp32)
        out = out + part.float()
    return out.double()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--c', type=int, default=128)
    ap.add_argument('--n', type=int, default=64)
    ap.add_argument('--hw', type=int, default=32)
    ap.add_argument('--seed', type=int, default=0)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(a.seed)
    C, N, S = a.c, a.n, a.hw
    z = torch.randn((C, S, S), generator=g, dtype=torch.float64) * 1.5 + 0.2
    x = z * torch.sigmoid(z)  # a GN + SiLU output
    w = torch.randn((N, C, 3, 3), generator=g, dtype=torch.float64) / (9 * C)**0.5
    xp = torch.nn.functional.pad(x, (1, 1, 1, 1))
    ref = torch.nn.functional.conv2d(xp[None], w)[0]  # [N][S][S]
    sa = pow2_scale(x.abs().max() * 2)  # the kernels' GN bound exponent, 1 bit of margin

    # direct: K = (tap, c)
    cols = torch.stack([xp[:, ky:ky + S, kx:kx + S] for ky in range(3) for kx in range(3)], 0)  # [9][C][S][S]
    A = cols.permute(2, 3, 0, 1).reshape(S * S, 9 * C) * sa
    Wm = w.permute(0, 2, 3, 1).reshape(N, 9 * C)
    sw = pow2_scale(Wm.abs().amax(1))
    y_dir = (f16x3_gemm(A, (Wm * sw[:, None]).t()) / sw[None, :] / sa).t().reshape(N, S, S)

    # 1D F(2,3) along x: per kernel row ky and position p, GEMM over channels
    Mx = torch.zeros((4, N, S, S // 2), dtype=torch.float64)
    sa1 = sa / 2  # |V| <= 2 max|d|
    for ky in range(3):
        rows = xp[:, ky:ky + S, :]  # [C][S][S+2]
        d = torch.stack([rows[:, :, j:j + S:2] for j in range(4)], -1)  # [C][S][S/2][4] windows of 4 at stride 2
        V = torch.einsum('pj,cyxj->pcyx', BT, d)  # [4][C][S][S/2]
        Uk = torch.einsum('pk,nck->pnc', G, w[:, :, ky, :])  # [4][N][C]
        swk = pow2_scale(Uk.abs().amax(dim=(0, 2)))  # per n over positions (and ky: the pack takes all)
        for p in range(4):
            Ap = V[p].permute(1, 2, 0).reshape(-1, C) * sa1
            Mx[p] += (f16x3_gemm(Ap, (Uk[p] * swk[:, None]).t()) / swk[None, :] / sa1).t().reshape(N, S, S // 2)
    y1d = torch.zeros((N, S, S), dtype=torch.float64)
    y1d[:, :, 0::2] = Mx[0] + Mx[1] + Mx[2]
    y1d[:, :, 1::2] = Mx[1] - Mx[2] - Mx[3]

    # 2D F(2x2,3x3): 16 positions per 2x2 output tile
    d2 = torch.stack([torch.stack([xp[:, i:i + S:2, j:j + S:2] for j in range(4)], -1) for i in range(4)], -2)  # [C][S/2][S/2][4][4]
    V2 = torch.einsum('pi,cyxij,qj->pqcyx', BT, d2, BT)  # [4][4][C][S/2][S/2]
    U2 = torch.einsum('pk,nckl,ql->pqnc', G, w, G)  # [4][4][N][C]
    sw2 = pow2_scale(U2.abs().amax(dim=(0, 1, 3)))
    sa2 = sa / 4  # |V2| <= 4 max|d|
    M2 = torch.zeros((4, 4, N, S // 2, S // 2), dtype=torch.float64)
    for p in range(4):
        for q in range(4):
            Ap = V2[p, q].permute(1, 2, 0).reshape(-1, C) * sa2
            M2[p, q] = (f16x3_gemm(Ap, (U2[p, q] * sw2[:, None]).t()) / sw2[None, :] / sa2).t().reshape(N, S // 2, S // 2)
    Y2 = torch.einsum('ip,pqnyx,jq->nyixj', AT, M2, AT)  # [N][S/2][2][S/2][2]
    y2d = Y2.reshape(N, S, S)

    def rel(y):
        return float((y - ref).norm() / ref.norm())

    print(f'C={C} N={N} {S}x{S}: rel-L2 vs float64  direct {rel(y_dir):.2e}  wino-1D {rel(y1d):.2e}  '
          f'wino-2D {rel(y2d):.2e}')


if __name__ == '__main__':
    main()
