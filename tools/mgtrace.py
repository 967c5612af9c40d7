"""MoGAN C5 optimize_parameters calls (B=1, 1024x436) for a kernel trace (rocprofv3 --kernel-trace --stats --
python3 tools/mgtrace.py): 2 warm-up calls, then `steps` traced calls (E and M alternating)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main(steps=4, B=1, H=436, W=1024):
    from gbvst import _lib, mogan_model
    from gbvst.options import default_opt
    _lib.load()
    dev = torch.device("cuda:0")
    opt = default_opt(True, model="mogan", pool_size=50, gpu_ids=[0])
    m = mogan_model.MoGANModel(opt)
    g = torch.Generator(device="cpu").manual_seed(3)
    m.set_input_fc2([(torch.rand(B, 3, H, W, generator=g) * 2 - 1) for _ in range(4)])
    for _ in range(2 + steps):
        m.optimize_parameters()
    torch.cuda.synchronize()
    print("steps", 2 + steps)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
