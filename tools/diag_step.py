"""Diagnostic: wc_ddpm_step vs the golden reference step at several t, with the golden tables."""
import numpy as np, torch, sys, os, struct
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
from weatherconverter_amd import kernels as K
g = np.load('tests/golden/sched.npz')
s = LinearNoiseScheduler(1000, 0.0001, 0.02)
for n in ('betas', 'alphas', 'alpha_cum_prod', 'sqrt_alpha_cum_prod', 'one_minus_cum_prod', 'sqrt_one_minus_alpha_cum_prod'):
    s._cpu[n] = torch.from_numpy(g[f'T1000_{n}'])
x = torch.from_numpy(g['step_xt']); e = torch.from_numpy(g['step_eps'])
hx = lambda f: struct.pack('>f', f).hex()
for t in (1, 37, 500, 999):
    b, s1m, sqa, sig = s.step_scalars(t)
    ref = g[f'step{t}_mean']
    out = torch.empty_like(x).cuda()
    K.ddpm_step(x.cuda(), e.cuda(), out, b, s1m, sqa, 0.0, mode=0)
    o = out.cpu().numpy()
    npx = (x.numpy() - (np.float32(b) * e.numpy()) / np.float32(s1m)) / np.float32(sqa)
    print(t, [hx(v) for v in (b, s1m, sqa)], 'kernel mism', int((o != ref).sum()), 'numpy-box mism', int((npx != ref).sum()),
          'kernel!=numpy', int((o != npx).sum()), 'sqrt check', hx(float(np.sqrt(np.float32(g['T1000_alphas'][t])))))
