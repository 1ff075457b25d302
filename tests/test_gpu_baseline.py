"""GPU parity at BASELINE.json's full sizes (configs 1-5, the exact bench.py workloads).

At these sizes the CPU oracle is too slow for the whole message, so each config is checked
three ways, all bit-exact:

* the whole packed stream against an independent closed-form gather of the same bytes
  (torch indexing of the user buffer on the GPU: the type map written out by hand from
  SURVEY.md §8d / Appendix A, not through either engine);
* the whole unpack into a 0xA5-filled buffer against the closed-form scatter: every
  type-map byte lands, every gap byte survives;
* the packed PREFIX that bench.py's cpu_baseline samples against the oracle
  (oracle/ddt_oracle.c, the restated reference convertor) run on the same input bytes.
"""
from __future__ import annotations

import numpy as np
import pytest

import bench
from . import recipes as R

pytestmark = pytest.mark.gpu


def _expected_units(name, torch, dev, fields=None):
    """(unit dtype, type-space unit indices of the packed stream in type-map order)."""
    if name == "cfg1":                      # vector(1024,1,2) double x 2048, extent 16376 B
        i = torch.arange(2048, device=dev, dtype=torch.int64)[:, None]
        j = torch.arange(1024, device=dev, dtype=torch.int64)[None, :]
        return torch.int64, (i * (16376 // 8) + 2 * j).reshape(-1)
    if name == "cfg2":                      # 6 faces of 256^3 double, 16 fields
        n = 256
        zy = torch.arange(n * n, device=dev, dtype=torch.int64)
        z = torch.arange(n, device=dev, dtype=torch.int64)[:, None]
        x = torch.arange(n, device=dev, dtype=torch.int64)[None, :]
        plane = torch.arange(n * n, device=dev, dtype=torch.int64)
        faces = [zy * n, zy * n + (n - 1),                                  # x-, x+
                 (z * n * n + x).reshape(-1), (z * n * n + (n - 1) * n + x).reshape(-1),
                 plane, (n - 1) * n * n + plane]                            # z-, z+
        one = torch.cat(faces)
        f = torch.arange(16, device=dev, dtype=torch.int64)[:, None]
        return torch.int64, (f * n ** 3 + one[None, :]).reshape(-1)
    if name == "cfg3":                      # 512^3 float subarray faces, start 511, 8 fields
        n = 512
        a = torch.arange(n, device=dev, dtype=torch.int64)
        faces = [(n - 1) * n * n + torch.arange(n * n, device=dev, dtype=torch.int64),
                 (a[:, None] * n * n + (n - 1) * n + a[None, :]).reshape(-1),
                 ((a[:, None] * n + a[None, :]) * n + (n - 1)).reshape(-1)]
        one = torch.cat(faces)
        f = torch.arange(fields or 8, device=dev, dtype=torch.int64)[:, None]
        return torch.int32, (f * n ** 3 + one[None, :]).reshape(-1)
    if name == "cfg4":                      # indexed_block(1, LCG disps) of float
        return torch.int32, torch.from_numpy(bench.lcg_disps(64 << 20)).to(dev)
    if name == "cfg5":                      # hvector(128Mi,1,32B) of struct{double,int[3]}
        k = torch.arange(128 << 20, device=dev, dtype=torch.int64)[:, None]
        return torch.int32, (k * 8 + torch.arange(5, device=dev, dtype=torch.int64)[None, :]).reshape(-1)
    raise AssertionError(name)


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4", "cfg5", "cfg3_64"])
def test_baseline_config_full_size(device, name):
    """cfg3_64: BASELINE config 3 as `bench.py --config cfg3 --strong` runs it on one GPU,
    all 64 fields (a 32 GiB user span: 64-bit offsets in every item)."""
    import torch
    import ompi_amd
    from ompi_amd import recipe as ER

    fields = None
    if name == "cfg3_64":
        name, fields = "cfg3", 64
    recipe, count, _ = bench.make_workload(name)
    count = fields or count
    dt = ER.build_committed(recipe)
    info = dt.info()
    S = info["size"] * count
    span, origin = bench.layout(info, count)
    g = torch.Generator(device=device)
    g.manual_seed(1234)
    user = torch.randint(1, 255, (span,), dtype=torch.uint8, device=device, generator=g)
    packed = torch.zeros(S, dtype=torch.uint8, device=device)
    assert ompi_amd.pack(user.data_ptr() + origin, count, dt, packed, S, 0) == S

    ut, idx = _expected_units(name, torch, device, fields)
    unit = torch.tensor([], dtype=ut).element_size()
    assert idx.numel() * unit == S
    assert origin % unit == 0 and span % unit == 0
    idx = idx + origin // unit              # type-space units -> buffer units (true_lb shift)
    assert int(idx.min()) >= 0 and int(idx.max()) < span // unit
    uw = user.view(ut)
    pw = packed.view(ut)
    assert torch.equal(pw, uw[idx]), f"{name}: packed stream differs from the closed-form gather"

    # the prefix bench.py's cpu_baseline samples, against the oracle on the same bytes
    srec, scount, _ = bench.sample_recipe(name, recipe, count)
    b = R.Built(srec)
    si = b.o.info()
    sext = si["ub"] - si["lb"]
    hi = max(si["true_ub"], si["true_ub"] + (scount - 1) * sext)
    host = user[:min(span, origin + hi)].cpu().numpy()
    ref = np.frombuffer(b.o.pack_all(scount, host, origin), dtype=np.uint8)
    np.testing.assert_array_equal(packed[:ref.size].cpu().numpy(), ref)
    del host, ref

    # unpack into a sentinel-filled buffer: type-map bytes land, gap bytes survive
    del user
    out = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
    assert ompi_amd.unpack(packed, S, 0, out.data_ptr() + origin, count, dt) == S
    exp = torch.full((span,), 0xA5, dtype=torch.uint8, device=device)
    exp.view(ut)[idx] = pw
    torch.cuda.synchronize()
    assert torch.equal(out, exp), f"{name}: unpacked buffer differs from the closed-form scatter"
