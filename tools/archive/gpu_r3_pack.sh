#!/bin/bash
# the device pack test alone, plus the same check torch-GPU vs torch-CPU (diagnostic)
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 120 --timeout-method thread -k device_pack > gpurun_out/pack_tests.log 2>&1
rc=$?; echo rc=$rc; grep -E "PASS|FAIL|differ" gpurun_out/pack_tests.log | head -30
timeout -k 10 100 python -u - > gpurun_out/pack_diag.log 2>&1 <<'PY'
import torch
from weatherconverter_amd import kernels as K
g = torch.Generator().manual_seed(12)
w = torch.randn((128, 576), generator=g) * torch.exp(torch.randn((128, 1), generator=g) * 3)
a = K.pack_f16x3(w.cuda(), 64, 0, device=False).data.cpu()
b = K.pack_f16x3(w, 64, 0, device=False).data
c = K.pack_f16x3(w.cuda(), 64, 0, device=True).data.cpu()
print('torchGPU==torchCPU', torch.equal(a, b), int((a != b).sum()), 'dev==torchCPU', torch.equal(c, b), int((c != b).sum()),
      'dev==torchGPU', torch.equal(c, a), int((c != a).sum()))
d = (c != b).flatten().nonzero()[:5].flatten().tolist()
print([(i, int(c.flatten()[i]), int(b.flatten()[i])) for i in d])
PY
cat gpurun_out/pack_diag.log
exit $rc
