"""CPU checks of the op layer: weight packing layouts and the reference paths."""
import math

import torch

from vgate import ops
from vgate.ops import reference as ref


def test_pack_roundtrip_and_fragment_layout():
    N, K = 48, 96
    w = torch.randn(N, K).bfloat16()
    wp = ops.pack_weight(w)
    assert torch.equal(ops.unpack_weight(wp, N, K), w)
    flat = wp.reshape(-1, 8)
    # tile (nt=1, kt=2), lane 37 -> row 16 + 37%16, cols 64 + 8*(37//16) ...
    nt, kt, lane = 1, 2, 37
    idx = (nt * (K // 32) + kt) * 64 + lane
    assert torch.equal(flat[idx], w[16 * nt + lane % 16, 32 * kt + 8 * (lane // 16): 32 * kt + 8 * (lane // 16) + 8])


def test_interleave_gate_up_roundtrip():
    I, K = 64, 32
    wg, wu = torch.randn(I, K).bfloat16(), torch.randn(I, K).bfloat16()
    lin = ops.Linear(torch.cat([wg, wu]), kind="silu")
    assert torch.equal(lin.dense_weight(), torch.cat([wg, wu]))
    x = torch.randn(3, K).bfloat16()
    assert torch.allclose(ops.linear(x, lin).float(), ref.silu_mul_linear_ref(x, wg, wu).float())


def test_pack_awq_layout():
    N, K = 32, 256
    q = torch.randint(0, 16, (N, K), dtype=torch.int32)
    p = ops.pack_awq(q).view(torch.int32).reshape(-1)
    nt, kq, lane, u = 1, 1, 21, 2
    word = int(p[((nt * (K // 128) + kq) * 64 + lane) * 4 + u]) & 0xFFFFFFFF
    row = 16 * nt + (lane & 15)
    k0 = 128 * kq + 32 * u + 8 * (lane >> 4)
    # value j at bit (16 if j odd) + 4 (j >> 1): (word >> 4d) & 0x000F000F holds values 2d, 2d+1
    vals = [(word >> ((j & 1) * 16 + 4 * (j >> 1))) & 0xF for j in range(8)]
    assert vals == q[row, k0:k0 + 8].tolist()
    for d in range(4):
        pair = ((word >> (4 * d)) & 0x000F000F) | 0x43004300
        lo = torch.tensor([pair & 0xFFFF], dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
        hi = torch.tensor([(pair >> 16) & 0xFFFF], dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
        assert lo.item() == 128 + vals[2 * d] and hi.item() == 128 + vals[2 * d + 1]


def test_attention_ref_matches_dense():
    torch.manual_seed(0)
    Hq, Hkv, D, BS = 4, 2, 128, 16
    ctx = 40
    kc = torch.randn(8, Hkv, BS, D).bfloat16()
    vc = torch.randn(8, Hkv, BS, D).bfloat16()
    bt = torch.tensor([[5, 2, 7, 0]], dtype=torch.int32)
    q = torch.randn(1, Hq, D).bfloat16()
    out = ref.attention_ref(q, kc, vc, bt, torch.tensor([ctx]), torch.tensor([0, 1]), Hq, Hkv, 1 / math.sqrt(D))
    K = torch.cat([kc[b] for b in [5, 2, 7]], dim=1)[:, :ctx].float()
    V = torch.cat([vc[b] for b in [5, 2, 7]], dim=1)[:, :ctx].float()
    for h in range(Hq):
        kv = h // 2
        p = torch.softmax(q[0, h].float() @ K[kv].t() / math.sqrt(D), -1)
        assert torch.allclose(out[0, h].float(), (p @ V[kv]), atol=2e-2)


def test_rope_table_llama3_scaling_shapes():
    t = ref.rope_cos_sin(64, 128, 5e5, {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                         "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    assert t.shape == (64, 128)
    assert torch.allclose(t[0, :64], torch.ones(64))


def test_sample_ref_topk():
    logits = torch.tensor([[0.0, 5.0, 1.0, 4.0]])
    gens = [torch.Generator().manual_seed(0)]
    outs = {int(ref.sample_ref(logits, torch.tensor([1.0]), None, torch.tensor([2]), gens)[0]) for _ in range(50)}
    assert outs <= {1, 3}


def test_native_allocator_if_built():
    try:
        C = ops.native()
    except RuntimeError:
        import pytest
        pytest.skip("native extension not built")
    a = C.BlockAllocator(8, 16, True)
    b = a.allocate(3)
    assert len(set(b)) == 3 and a.num_free() == 5
    h = C.BlockAllocator.hash_block(0, [1, 2, 3])
    a.register_hash(b[0], h)
    a.free(b)
    assert a.num_free() == 8
    got = a.lookup(h)
    assert got == b[0] and a.refcount(got) == 1 and a.num_free() == 7
    a.free([got])
    # evictable cached block is reused last
    c = a.allocate(8)
    assert len(set(c)) == 8
    assert a.lookup(h) == -1


def test_unpack_awq_inverts_pack():
    torch.manual_seed(3)
    q = torch.randint(0, 16, (48, 384), dtype=torch.int32)
    assert torch.equal(ops.unpack_awq(ops.pack_awq(q), 48, 384), q)


def test_prefill_plan_bucket_lookup():
    """A step's rows are padded up to its graph bucket: the plan of the smallest planned M >= M
    applies; larger M than any planned bucket keeps the launcher's heuristic (None)."""
    plan = {128: (128, 0), 384: (128, 4), 512: (1024, 0)}
    assert ops._plan_bucket(plan, 128) == 128
    assert ops._plan_bucket(plan, 200) == 384
    assert ops._plan_bucket(plan, 512) == 512
    assert ops._plan_bucket(plan, 513) is None
    assert ops._plan_bucket({}, 64) is None


def test_tune_prefill_without_gpu_is_a_no_op():
    lin = ops.Linear(torch.randn(64, 64).bfloat16())
    assert ops.tune_prefill([lin], [128, 256]) == {}
    assert lin.prefill_plan == {}


def test_host_device_copy_cpu_fallback():
    """Without a GPU tensor the helper is a plain prefix copy (the CPU engine's path)."""
    src = torch.arange(64, dtype=torch.int32)
    dst = torch.zeros(64, dtype=torch.int32)
    ops.host_device_copy(dst, src, 40)
    assert torch.equal(dst[:10], src[:10]) and int(dst[10:].abs().sum()) == 0


def test_plan_cache_round_trip(tmp_path):
    """Persisted start-up GEMM plans: stored per key, other keys kept, tuples restored."""
    from vgate import ops
    path = str(tmp_path / "sub" / "plans.json")
    plans = {(2048, 1536): {128: (128, 0), 48: (-1, -1)}, (17920, 1536): {512: (768, 2)}}
    assert ops.load_plan_cache(path, "k1") is None
    ops.save_plan_cache(path, "k1", plans)
    ops.save_plan_cache(path, "k2", {(1, 2): {3: (4, 5)}})
    assert ops.load_plan_cache(path, "k1") == plans
    assert ops.load_plan_cache(path, "k2") == {(1, 2): {3: (4, 5)}}
    assert ops.load_plan_cache(path, "nope") is None


def test_decode_plans_apply_tile_and_streamk_entries():
    """decode_plans.apply sets tile-kernel plans on (waves, K slices, tiles) and stream-K plans on
    ("sk", waves, blocks per CU, group) entries, by (N, K, layout, kind)."""
    from types import SimpleNamespace
    from vgate.models import decode_plans

    def lin(N, K, layout="plain", kind="dense"):
        return SimpleNamespace(N=N, K=K, layout=layout, kind=kind, dec_waves=0, dec_splitk=0, dec_ntb=0, dec_sk=None)
    L = SimpleNamespace(qkv=lin(6144, 4096, "qkv"), o=lin(4096, 4096), gate_up=lin(28672, 4096, "silu"),
                        down=lin(4096, 14336))
    model = SimpleNamespace(layers=[L], lm_head=lin(128256, 4096))
    n = decode_plans.apply(model)
    assert n == 3
    assert L.qkv.dec_sk == (8, 1, 4) and L.qkv.dec_waves == 0
    assert (L.gate_up.dec_waves, L.gate_up.dec_splitk, L.gate_up.dec_ntb) == (4, 1, 0) and L.gate_up.dec_sk is None
    assert (L.down.dec_waves, L.down.dec_splitk, L.down.dec_ntb) == (4, 1, 1)
    assert L.o.dec_sk is None and L.o.dec_waves == 0
    for key, val in decode_plans.PLANS.items():
        assert len(key) == 4 and key[2] in ("qkv", "silu", "plain") and key[3] in ("dense", "awq")
        assert (val[0] in ("sk", "kx") and len(val) == 4) or (len(val) == 3 and all(isinstance(v, int) for v in val))
    # a register-stationary entry selects decode path 4 with its (waves, slices, tiles code)
    kxl = lin(17920, 1536, "silu")
    kxl.dec_path = 0
    decode_plans.apply(SimpleNamespace(layers=[SimpleNamespace(qkv=lin(1, 1), o=lin(1, 1), gate_up=kxl, down=lin(1, 1))],
                                       lm_head=lin(1, 1)))
    assert kxl.dec_path == 4 and (kxl.dec_waves, kxl.dec_splitk, kxl.dec_ntb) == (0, 0, 0)


def test_linear_qkv_with_attention_cpu():
    """ops.linear(qkv=..., attn=...) on the CPU: the projection, RoPE + KV write, then the decode
    attention over its q (the GPU runs both in one launch, csrc/kernels/qkv_attn.hip)."""
    torch.manual_seed(3)
    S, H, D, BS, hq, hkv = 3, 256, 128, 16, 4, 2
    N = (hq + 2 * hkv) * D
    lin = ops.Linear((torch.randn(N, H) / H ** 0.5).bfloat16(), layout="qkv")
    x = torch.randn(S, H).bfloat16()
    bt = torch.arange(S * 4, dtype=torch.int32).view(S, 4)
    kc = torch.randn(S * 4, hkv, BS, D).bfloat16()
    vc = torch.randn(S * 4, hkv, BS, D).bfloat16()
    cl = torch.tensor([5, 17, 40], dtype=torch.int32)
    pos = cl - 1
    slots = (bt[torch.arange(S), (pos // BS).long()] * BS + pos % BS).int()
    qs = torch.arange(S + 1, dtype=torch.int32)
    cs = ref.rope_cos_sin(64, D, 1e4)
    qkv = dict(positions=pos, slots=slots, cos_sin=cs, k_cache=kc, v_cache=vc, hq=hq, hkv=hkv)
    o = torch.zeros(S, hq * D).bfloat16()
    part_o = torch.empty(S, hq, 1, D)
    part_ml = torch.empty(S, hq, 1, 2)
    q = ops.linear(x, lin, qkv=qkv, attn=dict(block_tables=bt, context_lens=cl, query_start=qs, out=o,
                                              part_o=part_o, part_ml=part_ml, part_size=64, scale=D ** -0.5))
    ro = ref.attention_ref(q.view(S, hq, D), kc, vc, bt, cl, qs, hq, hkv, D ** -0.5).view(S, hq * D)
    assert torch.allclose(o.float(), ro.float(), atol=2e-2, rtol=2e-2)
    # the new token's K row was written before the attention read it
    assert torch.count_nonzero(o.float()) > 0
