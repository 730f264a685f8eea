import torch, sys, os
sys.path.insert(0, os.getcwd())
from aiforearth_api_platform_amd.ops.conv import pack_conv, pack_stem_s2d, stem_pool_c1, stem_pool_c1_u8, conv2d_nhwc
from aiforearth_api_platform_amd.ops.pool import preprocess_s2d_u8
g = torch.Generator().manual_seed(1)
w7 = torch.randn(64, 3, 7, 7, generator=g) / 12
b = torch.randn(64, generator=g) * 0.1
w1 = torch.randn(64, 64, 1, 1, generator=g) / 8
b1 = torch.randn(64, generator=g) * 0.1
pc = pack_stem_s2d(w7, b).to("cuda"); c1 = pack_conv(w1, b1).to("cuda")
for shape in [(2, 64, 96), (3, 224, 224)]:
    img = torch.randint(0, 256, (*shape, 3), dtype=torch.uint8, device="cuda")
    y, t1 = stem_pool_c1_u8(img, pc, c1)
    t1y = conv2d_nhwc(y, c1, relu=True)
    d = (t1.float() - t1y.float()).abs()
    idx = (d == d.max()).nonzero()[:5].tolist()
    print(shape, "t1 vs conv(y):", d.max().item(), idx, "count>0.1:", (d > 0.1).sum().item(), flush=True)
    y2, t12 = stem_pool_c1(preprocess_s2d_u8(img), pc, c1)
    d2 = (t12.float() - conv2d_nhwc(y2, c1, relu=True).float()).abs()
    print(shape, "old path t1 vs conv(y):", d2.max().item(), flush=True)
