"""Dev tool (GPU): the fused loss + gradient (lt_loss_grad, one launch for the
bigram) against lt_loss_forward + lt_loss_backward with checkpoints, on the
BASELINE shape and a few edge shapes, with the workspace poisoned (NaN bytes)
before every call so a stale hand-off read shows; then timings."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from last_torch_amd import _native as nat  # noqa: E402


def ref(W, nf, lab, nl, V, n, local):
  out = nat.loss_forward(W, nf, lab, nl, V, n, local, checkpoints=True)
  dW = nat.loss_backward(W, nf, lab, nl, *out[1:5], None, V, n, local, ck=out[5])
  return out[0], dW


def check(B, T, U, V, n=1, bf16=False, local=False, varlen=True, seed=0):
  g = torch.Generator(device='cuda')
  g.manual_seed(seed)
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], generator=g, device='cuda')
  if bf16:
    W = W.bfloat16()
  if local:
    W = torch.log_softmax(W.float(), -1).to(W.dtype)
  nf = (torch.randint(T // 2, T + 1, [B], generator=g, device='cuda', dtype=torch.int32)
        if varlen else torch.full([B], T, dtype=torch.int32, device='cuda'))
  nf[0] = T
  lab = torch.randint(1, V + 1, [B, U], generator=g, device='cuda', dtype=torch.int32)
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  if B > 2:
    nl[1] = U + 5   # unreachable: loss +inf, dW 0
    lab[2, ::3] = 0  # epsilons
  r_loss, r_dW = ref(W, nf, lab, nl, V, n, local)
  ws_bytes = nat.ctypes.c_size_t()
  pb = nat._problem(W, V, n, U)
  nat._check(nat.lib().lt_loss_grad_workspace_bytes(nat.ctypes.byref(pb), int(local),
                                                    nat.ctypes.byref(ws_bytes)), 'ws')
  ws = torch.full([ws_bytes.value], 0xFF, dtype=torch.uint8, device='cuda')
  loss, _, _, dW = nat.loss_grad(W, nf, lab, nl, V, n, local, workspace=ws)
  torch.cuda.synchronize()
  err = nat.grad_workspace_errors(ws, W, V, n, U, local)
  fin = torch.isfinite(r_loss)
  same_inf = bool((torch.isfinite(loss) == fin).all())
  dl = float((loss - r_loss)[fin].abs().max()) if fin.any() else 0.0
  dd = (dW.float() - r_dW.float()).abs()
  tol = 1e-5 + 2e-6 * r_loss.abs().clamp(min=1, max=1e6)
  rel = float((dd.reshape(B, -1).max(1).values / tol.where(fin, torch.ones_like(tol))).max())
  nan = bool(torch.isnan(dW).any())
  lmax = float(r_loss[fin].abs().max()) if fin.any() else 0.0
  ok = same_inf and err == 0 and not nan and dl <= 1e-5 + 1e-6 * lmax
  print(f'B={B} T={T} U={U} V={V} bf16={bf16} local={local}: loss max|d| {dl:.2e} '
        f'dW max|d| {float(dd.max()):.2e} (x tol {rel:.2f}) nan={nan} err={err} '
        f'inf-equal={same_inf} {"OK" if ok else "FAIL"}', flush=True)
  return ok


def timeit(fn, reps=20):
  fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
  e0.record()
  for _ in range(reps):
    fn()
  e1.record()
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) / reps


def main():
  ok = True
  ok &= check(4, 40, 6, 5)
  ok &= check(8, 100, 10, 32)
  ok &= check(8, 100, 10, 32, bf16=True)
  ok &= check(8, 100, 10, 32, local=True)
  ok &= check(16, 300, 40, 8)
  ok &= check(5, 77, 3, 2)
  ok &= check(3, 1, 2, 4)
  ok &= check(64, 1000, 100, 32, varlen=False)
  ok &= check(64, 1000, 100, 32, bf16=True)
  ok &= check(100, 500, 200, 32)
  print('ALL OK' if ok else 'SOME FAILED', flush=True)
  B, T, U, V, n = 64, 1000, 100, 32, 1
  C = nat.num_context_states(V, n)
  W = torch.randn([B, T, C, V + 1], device='cuda')
  nf = torch.full([B], T, dtype=torch.int32, device='cuda')
  lab = torch.randint(1, V + 1, (B, U), dtype=torch.int32, device='cuda')
  nl = torch.full([B], U, dtype=torch.int32, device='cuda')
  g1 = torch.ones([B], device='cuda')
  ws = torch.empty([1 << 30], dtype=torch.uint8, device='cuda')
  t_ref = timeit(lambda: ref(W, nf, lab, nl, V, n, False))
  for marg in os.environ.get('MARG', '').split(',') if os.environ.get('MARG') else ['']:
    if marg:
      os.environ['LT_FUSED_MARG'] = marg
    t_f = timeit(lambda: nat.scale_grad(nat.loss_grad(W, nf, lab, nl, V, n, False,
                                                      workspace=ws)[3], g1, V, n))
    print(f'marg={marg or "default"}: fused {t_f:.3f} ms  (fwd+bwd checkpoints {t_ref:.3f} ms)',
          flush=True)
  if not ok:
    sys.exit(1)


if __name__ == '__main__':
  main()
