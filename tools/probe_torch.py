import torch  # torch first: its HIP runtime becomes the process runtime
import numpy as np, sys
sys.path.insert(0, '.')
from vitpkg import vit
assert vit.lib().vit_init(0) == 0
a = vit.DeviceArray.from_numpy(np.ones(10, np.float32)); b = vit.DeviceArray.from_numpy(np.full(10, 2, np.float32)); o = vit.DeviceArray.zeros(10, np.float32)
vit.call("residual_forward", o, a, b, 10)
print("torch-first residual:", o.numpy()[:3], torch.cuda.is_available(), torch.version.hip)
t = torch.ones(4, device="cuda")
vit.call("residual_forward", vit.DeviceArray.zeros(1, np.float32), a, b, 1)
torch.cuda.synchronize(); print("torch tensor ok", t.sum().item())
