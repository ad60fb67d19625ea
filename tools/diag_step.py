"""Diagnostic: where does wc_ddpm_step differ from the reference's fp32 torch chain?"""
import numpy as np, torch, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from weatherconverter_amd.diffusion_model.scheduler.linear_noise_scheduler import LinearNoiseScheduler
from weatherconverter_amd import kernels as K
g = np.load('tests/golden/sched.npz')
s = LinearNoiseScheduler(1000, 0.0001, 0.02)
x = torch.from_numpy(g['step_xt']); e = torch.from_numpy(g['step_eps'])
for t in (1, 37, 500):
    b, s1m, sqa, sig = s.step_scalars(t)
    ref = g[f'step{t}_mean']
    out = torch.empty_like(x).cuda(); sz = torch.empty_like(out)
    K.ddpm_step(x.cuda(), e.cuda(), out, b, s1m, sqa, sig, z=torch.zeros_like(x).cuda(), mode=1, sz_out=sz)
    o = out.cpu().numpy()
    out2 = torch.empty_like(x).cuda()
    K.ddpm_step(x.cuda(), e.cuda(), out2, b, s1m, sqa, 0.0, mode=0)
    gt = ((x.cuda() - (b * e.cuda()) / s1m) / sqa).cpu().numpy()
    npx = (x.numpy() - (np.float32(b) * e.numpy()) / np.float32(s1m)) / np.float32(sqa)
    bad = np.nonzero(o.ravel() != ref.ravel())[0]
    print(t, 'kernel(sz) mism', len(bad), 'kernel(nonoise) mism', int((out2.cpu().numpy() != ref).sum()),
          'torchgpu mism', int((gt != ref).sum()), 'numpy mism', int((npx != ref).sum()))
    for i in bad[:3]:
        print('  idx', i, 'x', x.numpy().ravel()[i], 'e', e.numpy().ravel()[i], 'k', o.ravel()[i], 'ref', ref.ravel()[i])
