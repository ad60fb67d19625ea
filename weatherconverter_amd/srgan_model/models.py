"""Swift-SRGAN x4 generator with the reference's parameter tree (``srgan_model/models.py:1-92``).

It runs every guided step (``translation.py:81``) between the 128-px diffusion space and the 512-px
segmenter.  PyTorch-ROCm here (SURVEY §8(f) "next" #2 lists its depthwise convs as a later HIP target);
state_dict keys match the reference so its ``{'model': ...}`` checkpoints load.
"""
import torch
from torch import nn


class SeperableConv2d(nn.Module):  # (sic) reference spelling, keeps the key names

    def __init__(self, cin, cout, kernel_size, stride=1, padding=1, bias=True):
        super().__init__()
        self.depthwise = nn.Conv2d(cin, cin, kernel_size, stride=stride, padding=padding, groups=cin, bias=bias)
        self.pointwise = nn.Conv2d(cin, cout, 1, bias=bias)

    def forward(self, x):
        return self.pointwise(self.depthwise(x))


class ConvBlock(nn.Module):

    def __init__(self, cin, cout, use_act=True, use_bn=True, discriminator=False, **kw):
        super().__init__()
        self.use_act = use_act
        self.cnn = SeperableConv2d(cin, cout, **kw, bias=not use_bn)
        self.bn = nn.BatchNorm2d(cout) if use_bn else nn.Identity()
        self.act = nn.LeakyReLU(0.2, inplace=True) if discriminator else nn.PReLU(num_parameters=cout)

    def forward(self, x):
        y = self.bn(self.cnn(x))
        return self.act(y) if self.use_act else y


class UpsampleBlock(nn.Module):

    def __init__(self, cin, scale_factor):
        super().__init__()
        self.conv = SeperableConv2d(cin, cin * scale_factor**2, kernel_size=3, stride=1, padding=1)
        self.ps = nn.PixelShuffle(scale_factor)
        self.act = nn.PReLU(num_parameters=cin)

    def forward(self, x):
        return self.act(self.ps(self.conv(x)))


class ResidualBlock(nn.Module):

    def __init__(self, c):
        super().__init__()
        self.block1 = ConvBlock(c, c, kernel_size=3, stride=1, padding=1)
        self.block2 = ConvBlock(c, c, kernel_size=3, stride=1, padding=1, use_act=False)

    def forward(self, x):
        return self.block2(self.block1(x)) + x


class Generator(nn.Module):
    """(tanh(final) + 1) / 2 output in [0, 1]; x4 by two PixelShuffle(2) stages."""

    def __init__(self, in_channels: int = 3, num_channels: int = 64, num_blocks: int = 16, upscale_factor: int = 4):
        super().__init__()
        self.initial = ConvBlock(in_channels, num_channels, kernel_size=9, stride=1, padding=4, use_bn=False)
        self.residual = nn.Sequential(*[ResidualBlock(num_channels) for _ in range(num_blocks)])
        self.convblock = ConvBlock(num_channels, num_channels, kernel_size=3, stride=1, padding=1, use_act=False)
        self.upsampler = nn.Sequential(*[UpsampleBlock(num_channels, 2) for _ in range(upscale_factor // 2)])
        self.final_conv = SeperableConv2d(num_channels, in_channels, kernel_size=9, stride=1, padding=4)

    def forward(self, x):
        initial = self.initial(x)
        x = self.convblock(self.residual(initial)) + initial
        return (torch.tanh(self.final_conv(self.upsampler(x))) + 1) / 2


def load_model(model_path: str, device=None) -> nn.Module:
    """reference srgan_model/inference.py:9-16 (weights_only checkpoint load)."""
    device = device or torch.device('cuda' if torch.cuda.is_available() else 'cpu')
    net = Generator(upscale_factor=4).to(device)
    net.load_state_dict(torch.load(model_path, map_location=device, weights_only=True)['model'])
    return net.eval()


@torch.no_grad()
def inference(netG: nn.Module, lr_image: torch.Tensor) -> torch.Tensor:
    """reference srgan_model/inference.py:35-39."""
    return netG(lr_image)
