"""Profile-friendly DIP step loop: N training steps of one net/size without the ISTA side.

python tools/prof_dip_step.py unet1lip|skip C H W steps"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lrs-pnp-dip_amd"))
from lrspnp.dip import DipNet, lipschitz_unet_nodes, skip_nodes  # noqa: E402

net, C, H, W, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
n = DipNet(lipschitz_unet_nodes(C, C) if net == "unet1lip" else skip_nodes(C, C), C, H, W)
n.init_params(1)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.rand(C, H, W, device="cuda", generator=g)
t = torch.rand(n.out_shape, device="cuda", generator=g)
m = (torch.rand(n.out_shape[1:], device="cuda", generator=g) > 0.2).float()
n.train_steps(x, t, m, steps, use_graph=False)   # eager, as the bench (DipConfig.use_graph = False)
torch.cuda.synchronize()
print("loss", n.last_loss())
