"""CPU oracle for the learning-based style path and the RAFT correlation.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): stock-PyTorch CPU (NCHW fp32) restatements of
the reference arithmetic, checked against fixtures the reference itself produced
(oracle/gen_golden_style.py -> tests/golden/style_small.npz, corr_small.npz) by
tests/test_oracle_golden.py, then used as the checker of the HIP path.

Reference files restated (paths relative to the reference root):
  methods/learning-based/fs_lib.py:5-39                 warp (grid_sample * validity mask)
  methods/learning-based/network.py:10-78               Vgg16 / Vgg19 slices over torchvision's
                                                        VGG `features` (cfg D / E, 3x3 conv + ReLU,
                                                        MaxPool2d(2, 2))
  methods/learning-based/network.py:95-298              ConvLayer, ConvTanh, ConvInstRelu,
                                                        UpsampleConvInstRelu, ResidualBlock,
                                                        FastStyleNet (n_styles = 1)
  methods/learning-based/fast_style_transfer.py:795-822 calc_tv_loss, gram_matrix, normalize
  methods/learning-based/fs_johnson.py:25-47            Johnson.train_method losses
  utils/raft/raft/corr.py:12-60 + utils/utils.py:57-71  CorrBlock, bilinear_sampler
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

VGG_CFG = {
    "vgg16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "vgg19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
              512, 512, 512, 512, "M"],
}
VGG_SLICES = {"vgg16": [(0, 4), (4, 9), (9, 16), (16, 23)],
              "vgg19": [(0, 2), (2, 7), (7, 12), (12, 21), (21, 30)]}
VGG16_MEAN = [0.485, 0.456, 0.406]
VGG16_STD = [0.229, 0.224, 0.225]


# ------------------------------------------------------------------------------------ fs_lib
def fs_warp(x, flo):
    """fs_lib.py:5-39: grid_sample(x) * (grid_sample(ones) >= 0.9999), align_corners=False."""
    B, C, H, W = x.size()
    xx = torch.arange(0, W).view(1, -1).repeat(H, 1).view(1, 1, H, W).repeat(B, 1, 1, 1)
    yy = torch.arange(0, H).view(-1, 1).repeat(1, W).view(1, 1, H, W).repeat(B, 1, 1, 1)
    grid = torch.cat((xx, yy), 1).float()
    vgrid = grid + flo
    vx = 2.0 * vgrid[:, 0] / max(W - 1, 1) - 1.0
    vy = 2.0 * vgrid[:, 1] / max(H - 1, 1) - 1.0
    g = torch.stack([vx, vy], -1)
    out = F.grid_sample(x, g, align_corners=False)
    m = F.grid_sample(torch.ones_like(x), g, align_corners=False)
    m = torch.where(m < 0.9999, torch.zeros_like(m), m)
    m = torch.where(m > 0, torch.ones_like(m), m)
    return out * m


# --------------------------------------------------------------------------------------- VGG
def vgg_features(arch):
    """torchvision VGG `features` (cfg D / E) as an nn.Sequential."""
    layers, cin = [], 3
    for v in VGG_CFG[arch]:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return nn.Sequential(*layers)


class RefVGG(nn.Module):
    """network.py:10-78: slices of `features` with keys slice<k>.<feature index>."""

    def __init__(self, arch):
        super().__init__()
        feats = vgg_features(arch)
        self.arch = arch
        for k, (a, b) in enumerate(VGG_SLICES[arch]):
            s = nn.Sequential()
            for x in range(a, b):
                s.add_module(str(x), feats[x])
            setattr(self, "slice%d" % (k + 1), s)
        self.n = len(VGG_SLICES[arch])
        for p in self.parameters():
            p.requires_grad = False

    def forward(self, X):
        outs, h = [], X
        for k in range(self.n):
            h = getattr(self, "slice%d" % (k + 1))(h)
            outs.append(h)
        return tuple(outs)


# -------------------------------------------------------------------------------- FastStyleNet
class RefConvLayer(nn.Module):
    def __init__(self, cin, cout, k, stride):
        super().__init__()
        self.reflection_pad = nn.ReflectionPad2d(k // 2)
        self.conv2d = nn.Conv2d(cin, cout, k, stride=stride)

    def forward(self, x):
        return self.conv2d(self.reflection_pad(x))


class RefConvInstRelu(RefConvLayer):
    def __init__(self, cin, cout, k, stride):
        super().__init__(cin, cout, k, stride)
        self.instance = nn.InstanceNorm2d(cout, affine=True)

    def forward(self, x):
        return F.relu(self.instance(super().forward(x)))


class RefUpsampleConvInstRelu(nn.Module):
    def __init__(self, cin, cout, k):
        super().__init__()
        self.reflection_pad = nn.ReflectionPad2d(k // 2)
        self.conv2d = nn.Conv2d(cin, cout, k, 1)
        self.instance = nn.InstanceNorm2d(cout, affine=True)

    def forward(self, x):
        x = F.interpolate(x, scale_factor=2)
        return F.relu(self.instance(self.conv2d(self.reflection_pad(x))))


class RefResidualBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv1 = RefConvLayer(c, c, 3, 1)
        self.in1 = nn.InstanceNorm2d(c, affine=True)
        self.in2 = nn.InstanceNorm2d(c, affine=True)
        self.conv2 = RefConvLayer(c, c, 3, 1)
        self.layer_strength = nn.Parameter(torch.tensor([1], dtype=torch.float32))

    def forward(self, x, style_strength):
        s = style_strength * self.layer_strength
        s = 2 * s.abs() / (1 + s.abs())
        out = F.relu(self.in1(self.conv1(x)))
        out = self.in2(self.conv2(out))
        return s * out + x


class RefFastStyleNet(nn.Module):
    def __init__(self, num_inp=3):
        super().__init__()
        self.conv1 = RefConvInstRelu(num_inp, 32, 9, 1)
        self.conv2 = RefConvInstRelu(32, 64, 3, 2)
        self.conv3 = RefConvInstRelu(64, 128, 3, 2)
        for i in range(1, 6):
            setattr(self, "res%d" % i, RefResidualBlock(128))
        self.deconv1 = RefUpsampleConvInstRelu(128, 64, 3)
        self.deconv2 = RefUpsampleConvInstRelu(64, 32, 3)
        self.deconv3 = RefConvLayer(32, 3, 9, 1)

    def forward(self, x, style_strength=1.0):
        x = self.conv3(self.conv2(self.conv1(x)))
        for i in range(1, 6):
            x = getattr(self, "res%d" % i)(x, style_strength)
        feats = x
        x = self.deconv3(self.deconv2(self.deconv1(x)))
        return feats, torch.tanh(x / 255) * 150 + 255 / 2


# ------------------------------------------------------------------------------------- losses
def gram_matrix(inp):
    b, c, h, w = inp.size()
    f = inp.view(b, c, h * w)
    return torch.bmm(f, f.transpose(1, 2)).div(h * w)


def normalize(img):
    mean = img.new_tensor(VGG16_MEAN).view(-1, 1, 1)
    std = img.new_tensor(VGG16_STD).view(-1, 1, 1)
    return (img - mean) / std


def calc_tv_loss(I):
    sij = I[:, :, :-1, :-1]
    si1j = I[:, :, :-1, 1:]
    sij1 = I[:, :, 1:, :-1]
    tv1 = torch.norm(sij1 - sij, dim=1) ** 2
    tv2 = torch.norm(si1j - sij, dim=1) ** 2
    return torch.sum((tv1 + tv2) ** 0.5)


def johnson_losses(model, vgg, img, style_grams, alpha, beta, delta):
    """fs_johnson.py:25-47 train_method (single style): returns (loss, content, style, tv)."""
    _, styled = model(img)
    styled = styled / 255.0
    sf = vgg(normalize(styled))
    imf = vgg(normalize(img))
    content = alpha * F.mse_loss(sf[2], imf[2])
    style = 0
    for i, gs in enumerate(style_grams):
        style = style + ((gram_matrix(sf[i]) - gs) ** 2).mean()
    style = style * beta
    tv = delta * calc_tv_loss(styled)
    return content + style + tv, content, style, tv


# ------------------------------------------------------------------------------------- RAFT
def bilinear_sampler(img, coords):
    H, W = img.shape[-2:]
    xgrid, ygrid = coords.split([1, 1], dim=-1)
    xgrid = 2 * xgrid / (W - 1) - 1
    ygrid = 2 * ygrid / (H - 1) - 1
    grid = torch.cat([xgrid, ygrid], dim=-1)
    return F.grid_sample(img, grid, align_corners=True)


class RefCorrBlock:
    """corr.py:12-60."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        self.num_levels, self.radius = num_levels, radius
        b, d, h, w = fmap1.shape
        corr = torch.matmul(fmap1.view(b, d, h * w).transpose(1, 2), fmap2.view(b, d, h * w))
        # the reference's .float() (corr.py:22); dtype-following so the parity tests can run it in fp64
        corr = (corr / torch.sqrt(torch.tensor(d).to(fmap1.dtype))).reshape(b * h * w, 1, h, w)
        self.pyr = [corr]
        for _ in range(num_levels - 1):
            corr = F.avg_pool2d(corr, 2, stride=2)
            self.pyr.append(corr)

    def __call__(self, coords):
        r = self.radius
        coords = coords.permute(0, 2, 3, 1)
        b, h1, w1, _ = coords.shape
        outs = []
        for i in range(self.num_levels):
            d = torch.linspace(-r, r, 2 * r + 1, dtype=coords.dtype)
            delta = torch.stack(torch.meshgrid(d, d, indexing="ij"), axis=-1)
            c = coords.reshape(b * h1 * w1, 1, 1, 2) / 2 ** i + delta.view(1, 2 * r + 1, 2 * r + 1, 2)
            outs.append(bilinear_sampler(self.pyr[i], c).view(b, h1, w1, -1))
        return torch.cat(outs, dim=-1).permute(0, 3, 1, 2).contiguous().to(self.pyr[0].dtype)


def np_state(net):
    return {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}


# ------------------------------------------------------------------- fixture weights (PRNG)
def vgg_weights(net, base, init="fan_in"):
    """Counter-PRNG VGG state_dict.  init "fan_in": N(0, 2/fan_in) weights, N(0, 0.05) biases (the
    golden fixtures); "fan_out": torchvision's VGG init, kaiming_normal_(fan_out, relu) weights and
    zero biases — the scale the HIP model's own seeded Vgg16/Vgg19 use (perceptual.py)."""
    sd = {}
    for k, v in net.state_dict().items():
        if init == "fan_out":
            fan = int(v.shape[0] * np.prod(v.shape[2:])) if v.dim() > 1 else 1
            std = (2.0 / fan) ** 0.5
        else:
            fan = int(np.prod(v.shape[1:])) if v.dim() > 1 else 1
            std = (2.0 / fan) ** 0.5 if k.endswith("weight") else 0.05
        if init == "fan_out" and not k.endswith("weight"):
            sd[k] = np.zeros(tuple(v.shape), np.float32)
        else:
            sd[k] = _prng().normal(_prng().seed_for(k, base), tuple(v.shape), std=std)
    return sd


def fsn_weights(net, base):
    sd = {}
    for k, v in net.state_dict().items():
        shape, s = tuple(v.shape), _prng().seed_for(k, base)
        if k.endswith("layer_strength"):
            sd[k] = _prng().normal(s, shape, std=0.3, mean=1.0)
        elif ".instance." in k or ".in1." in k or ".in2." in k:
            sd[k] = _prng().normal(s, shape, std=0.1, mean=1.0 if k.endswith("weight") else 0.0)
        elif k.endswith("weight"):
            sd[k] = _prng().normal(s, shape, std=(1.0 / np.prod(shape[1:])) ** 0.5)
        else:
            sd[k] = _prng().normal(s, shape, std=0.02)
    return sd



def _prng():
    from oracle import prng
    return prng


def load_np(net, sd):
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return net
