import torch, sys
sys.path.insert(0, '/root/repo')
from gpu_mpi_tests_amd import ops
from gpu_mpi_tests_amd.ops import reference as ref
g = torch.Generator().manual_seed(6)
for (ny, nx) in [(33, 1030), (130, 516), (5, 255), (300, 640)]:
    z = torch.rand(ny + 4, nx, generator=g, dtype=torch.float64).cuda()
    out = ops.stencil5_2d(z, 1, scale=2.0)
    exp = ref.stencil5_2d(z.cpu(), 1, 2.0)
    bad = (out.cpu() - exp).abs() > 1e-12
    rows = bad.any(1).nonzero().flatten().tolist()
    cols = bad.any(0).nonzero().flatten().tolist()
    print(ny, nx, "bad", int(bad.sum()), "rows", rows[:10], "...", len(rows), "cols", cols[:5], "...", len(cols))
