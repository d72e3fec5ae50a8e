"""bench.py's roofline accounting (CPU): the algorithmic FLOPs and HBM bytes of a DIP training step,
checked by hand on a two-conv net and against the formula DESIGN.md §4 states for the 196^2 U-Net."""
import os
import sys
from types import SimpleNamespace as NS

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def _node(in0, cout, k, bn):
    return NS(kind=0, in0=in0, cout=cout, k=k, bn=bn)


def test_two_conv_net_by_hand():
    # input 3 x 8 x 8 -> conv 3x3 (BN) -> 4 x 8 x 8 -> conv 1x1 (no BN) -> 2 x 8 x 8
    net = NS(nodes=[_node(0, 4, 3, 1), _node(1, 2, 1, 0)], in_shape=(3, 8, 8), shapes=[(4, 8, 8), (2, 8, 8)],
             n_params=4 * 3 * 9 + 4 + 4 + 4 + 2 * 4 + 2)
    P = 64
    # conv 1 reads the network input: x once (forward) + once (weight gradient), z/y/BN 8 x out
    c1 = 3 * P + 8 * 4 * P
    # conv 2: 3 x its input (forward, data gradient out, weight gradient), 6 x out (no BN)
    c2 = 3 * 4 * P + 6 * 2 * P
    head = 3 * 2 * P
    assert bench.dip_alg_bytes_per_step(net) == 4 * (c1 + c2 + head + 7 * net.n_params)
    # FLOPs: forward + weight gradient for the input conv, + data gradient for the second
    f1 = 2 * 4 * 3 * 9 * P
    f2 = 2 * 2 * 4 * 1 * P
    assert bench.dip_flops_per_step(net) == 2 * f1 + 3 * f2


def test_unet_196_is_one_gigabyte_per_step():
    dims = [(128, 98), (128, 98), (128, 49), (128, 49), (128, 25), (128, 25), (128, 13), (128, 13), (128, 25),
            (128, 49), (128, 98), (128, 196), (128, 196), (198, 196)]
    ks = [3, 3, 3, 3, 3, 3, 3, 3, 2, 2, 3, 3, 1, 1]
    nodes = [_node(i, c, k, 0 if i == 13 else 1) for i, ((c, _), k) in enumerate(zip(dims, ks))]
    net = NS(nodes=nodes, in_shape=(198, 196, 196), shapes=[(c, h, h) for c, h in dims], n_params=434000)
    b = bench.dip_alg_bytes_per_step(net)
    assert 0.95e9 < b < 1.05e9, b


def test_cpu_baseline_host_fields():
    """The CPU baseline records the cores it used beside nproc, the machine's CPUs, the affinity set, the
    cgroup quota and the CPU model; by default it uses every CPU it may run on."""
    saved = os.environ.pop("OMP_NUM_THREADS", None)
    try:
        t = bench._threads()
        machine, aff, quota, model = bench.host_cpus()
        assert t == max(1, min(aff, int(quota)) if quota else aff)
        f = bench.host_fields(t)
        for k in ("cores", "nproc", "machine_cpus", "affinity_cpus", "cgroup_cpu_quota", "cpu_model"):
            assert k in f, k
        assert f["cores"] == t and f["machine_cpus"] == machine
    finally:
        if saved is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = saved
