"""Rounding budget of the checkpointing loss path (pipe_kernel -> marg_kernel)
at the BASELINE shape: the stored alpha / beta / alpha_num / beta_num rows,
log_z and num of a few utterances against a float64 numpy recursion, in units
of 2^-24 * max(1, |log_z|, |num|) (the per-element dW bound of
tests/golden_cases.marginal_scale allows 4 of them plus 1e-4 relative).
Also times nothing: a diagnostic for the round-4 precision work.

  python tools/ck_precision.py [utt ...]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from last_torch_amd import _native as nat  # noqa: E402


def lse(x, axis):
  m = np.max(x, axis=axis, keepdims=True)
  m = np.where(np.isfinite(m), m, 0.0)
  return np.squeeze(m, axis) + np.log(np.sum(np.exp(x - m), axis=axis))


def ref_bigram(W, nf, lab, nl):
  """float64 alpha [T,C], beta_{t+1} at frame t [T,C], log_z, alpha_num,
  beta_num (same convention), num for one bigram utterance."""
  T, C, R = W.shape
  W = W.astype(np.float64)
  al = np.full((T + 1, C), -np.inf)
  al[0, 0] = 0.0
  for t in range(nf):
    blank = al[t] + W[t, :, 0]
    lexq = lse(al[t][:, None] + W[t, :, 1:], axis=0)  # into q = y
    nxt = np.empty(C)
    nxt[0] = blank[0]
    nxt[1:] = np.logaddexp(blank[1:], lexq)
    al[t + 1] = nxt
  lz = lse(al[nf], axis=0)
  be = np.zeros((T + 1, C))
  for t in range(nf - 1, -1, -1):
    terms = np.concatenate([(W[t, :, 0] + be[t + 1])[:, None], W[t, :, 1:] + be[t + 1][None, 1:]],
                           axis=1)
    be[t] = lse(terms, axis=1)
  U = lab.shape[0]
  ctx = np.concatenate([[0], lab])
  an = np.full((T + 1, U + 1), -np.inf)
  an[0, 0] = 0.0
  for t in range(nf):
    stay = an[t] + W[t, ctx, 0]
    move = np.full(U + 1, -np.inf)
    move[1:] = an[t, :-1] + W[t, ctx[:-1], lab]
    an[t + 1] = np.logaddexp(stay, move)
  num = an[nf, nl]
  bn = np.full((T + 1, U + 1), -np.inf)
  bn[nf, nl] = 0.0
  for t in range(nf - 1, -1, -1):
    stay = W[t, ctx, 0] + bn[t + 1]
    move = np.full(U + 1, -np.inf)
    move[:-1] = W[t, ctx[:-1], lab] + bn[t + 1, 1:]
    bn[t] = np.logaddexp(stay, move)
  return al[:T], be[1:T + 1], lz, an[:T], bn[1:T + 1], num


def main():
  dev = torch.device('cuda', 0)
  B, T, U, V, n = 64, 1000, 100, 32, 1
  g = torch.Generator(device=dev)
  g.manual_seed(0)
  C = V + 1
  W = torch.randn([B, T, C, V + 1], generator=g, device=dev)
  nf = torch.randint(T // 2, T + 1, [B], generator=g, device=dev, dtype=torch.int32)
  nf[0] = T
  lab = torch.randint(1, V + 1, [B, U], generator=g, device=dev, dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device=dev)
  out = nat.loss_forward(W, nf, lab, nl, V, n, False, checkpoints=True)
  loss, lz, num, al, an, (be, bn, _) = out
  dW = nat.loss_backward(W, nf, lab, nl, lz, num, al, an, None, V, n, False, ck=out[5])
  torch.cuda.synchronize()
  utts = [int(x) for x in sys.argv[1:]] or [0, 1, 2]
  for b in utts:
    Wc = W[b].cpu().numpy()
    f = int(nf[b])
    ra, rb, rlz, ran, rbn, rnum = ref_bigram(Wc, f, lab[b].cpu().numpy(), int(nl[b]))
    unit = 2.0 ** -24 * max(1.0, abs(rlz), abs(rnum))

    def err(got, ref):
      got = got[:f].astype(np.float64)
      ref = ref[:f]
      fin = np.isfinite(ref)
      d = np.where(fin, np.abs(got - ref), 0.0)
      return d.max() / unit, d.mean() / unit

    print(f'utt {b} nf {f} log_z {rlz:.3f} (got {float(lz[b]):.4f}, err '
          f'{abs(float(lz[b]) - rlz) / unit:.2f} u) num {rnum:.3f} (err '
          f'{abs(float(num[b]) - rnum) / unit:.2f} u)')
    for name, got, ref in (('alpha', al[b], ra), ('beta', be[b], rb), ('alpha_num', an[b], ran),
                           ('beta_num', bn[b], rbn)):
      mx, mean = err(got.cpu().numpy(), ref)
      print(f'  {name:10s} max {mx:6.2f} u  mean {mean:6.2f} u')
    # den marginal exponents alpha + w + beta' - log_z against float64
    a64 = ra[:f, :, None]
    q = np.concatenate([np.arange(C)[:, None], np.tile(np.arange(1, C)[None, :], (C, 1))], axis=1)
    b64 = rb[:f][:, q]
    ex_ref = a64 + Wc[:f].astype(np.float64) + b64 - rlz
    ag = al[b].cpu().numpy()[:f].astype(np.float64)[:, :, None]
    bg = be[b].cpu().numpy()[:f].astype(np.float64)[:, q]
    ex_got = ag + Wc[:f].astype(np.float64) + bg - float(lz[b])
    live = ex_ref > -30
    d = np.abs(ex_got - ex_ref)[live]
    print(f'  den exponent (stored rows, exact arithmetic): max {d.max() / unit:6.2f} u '
          f'mean {d.mean() / unit:6.2f} u')
    # float64 den and string marginals, dW = den - num, and the kernel's dW
    # against them under golden_cases.marginal_scale
    den = np.exp(ex_ref)
    labc = lab[b].cpu().numpy()
    ctx = np.concatenate([[0], labc])
    U = labc.shape[0]
    nm = np.zeros_like(den)
    for t in range(f):
      eb = np.exp(ran[t] + Wc[t, ctx, 0] + rbn[t] - rnum)
      np.add.at(nm[t], (ctx, np.zeros(U + 1, np.int64)), np.where(np.isfinite(eb), eb, 0.0))
      el = np.exp(ran[t, :U] + Wc[t, ctx[:U], labc] + rbn[t, 1:] - rnum)
      np.add.at(nm[t], (ctx[:U], labc), np.where(np.isfinite(el), el, 0.0))
    ref = den - nm
    got = dW[b].cpu().numpy()[:f].astype(np.float64)
    scale = 1e-8 + (1e-4 + 4 * unit) * (den + nm)
    r = np.abs(got - ref) / scale
    i = np.unravel_index(np.argmax(r), r.shape)
    print(f'  dW / bound: max {r.max():.3f} at {list(i)} (den {den[i]:.3e} num {nm[i]:.3e}); '
          f'elements > 1: {(r > 1).sum()}')
    # the den and the num halves apart, relative to (den + num)
    tt, p_, y_ = i
    qq = q[p_, y_]
    dg = np.exp(np.float64(np.float32(al[b, tt, p_].item())) + Wc[tt, p_, y_] +
                np.float64(be[b, tt, qq].item()) - np.float64(lz[b].item()))
    print(f'    den from stored rows (exact arithmetic) err / (den+num): '
          f'{abs(dg - den[i]) / (den[i] + nm[i]):.3e}; total err / (den+num): '
          f'{abs(got[i] - ref[i]) / (den[i] + nm[i]):.3e}; 4 units: {4 * unit:.3e}')
    # the locally normalised loss: dW = -num marginals, bound relative to |num|
    outl = nat.loss_forward(W, nf, lab, nl, V, n, True, checkpoints=True)
    dWl = nat.loss_backward(W, nf, lab, nl, *outl[1:5], None, V, n, True, ck=outl[5])
    unl = 2.0 ** -24 * max(1.0, abs(rnum))
    gl = dWl[b].cpu().numpy()[:f].astype(np.float64)
    anl = outl[4][b].cpu().numpy()[:f].astype(np.float64)
    bnl = outl[5][1][b].cpu().numpy()[:f].astype(np.float64)
    ran_f, rbn_f = ran[:f], rbn[:f]
    print(f'  local: num err {abs(float(outl[2][b]) - rnum) / unl:.2f} un; alpha_num max '
          f'{np.abs(np.where(np.isfinite(ran_f), anl - ran_f, 0)).max() / unl:.2f} un, beta_num max '
          f'{np.abs(np.where(np.isfinite(rbn_f), bnl - rbn_f, 0)).max() / unl:.2f} un')
    rl = np.abs(gl + nm) / (1e-8 + (1e-4 + 4 * unl) * nm)
    il = np.unravel_index(np.argmax(rl), rl.shape)
    print(f'  local dW / bound: max {rl.max():.3f} at {list(il)} (num {nm[il]:.3e}); '
          f'> 1: {(rl > 1).sum()}')
    # string exponent errors at live string arcs (alpha_num + beta_num from
    # the stored rows, exact arithmetic)
    live = (ran_f + rbn_f - rnum) > -20
    e = np.abs((anl + bnl - float(outl[2][b])) - (ran_f + rbn_f - rnum))[live]
    print(f'  local string posterior exponent err: max {e.max() / unl:.2f} un mean {e.mean() / unl:.2f} un')


if __name__ == '__main__':
  main()
