"""Time to first token for long prompts (engine-level, one request at a time, after a
warm-up request of the same length so the step's hipGraph bucket is captured): prefill
throughput of the attention + GEMM kernels.

    python benchmarks/ttft_probe.py --model Qwen/Qwen2.5-1.5B-Instruct --lens 512 2048 4096
"""
import argparse
import json
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from vgate.runtime.engine import EngineConfig, LLMEngine  # noqa: E402
from vgate.runtime.sampling_params import SamplingParams  # noqa: E402


def one(eng, rid, ids):
    ev = threading.Event()
    out = {}

    def cb(kind, seq, payload):
        if kind != "token":
            out["ttft"] = seq.first_token_time - seq.arrival
            ev.set()

    eng.add_request(rid, params=SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True), callback=cb,
                    prompt_ids=ids)
    ev.wait(600)
    return out["ttft"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="Qwen/Qwen2.5-1.5B-Instruct")
    ap.add_argument("--lens", type=int, nargs="+", default=[512, 2048, 4096])
    ap.add_argument("--chunk", type=int, default=2048)
    ap.add_argument("--quantization", default=None)
    ap.add_argument("--shared-prefix", action="store_true",
                    help="the rounds 3-6 prompts: every length's prompt starts with the shorter ones' (prefix-cache hits)")
    a = ap.parse_args()
    eng = LLMEngine(EngineConfig(model=a.model, max_model_len=max(a.lens) + 16, max_num_seqs=16,
                                 max_num_batched_tokens=a.chunk, num_kv_blocks=4096,
                                 quantization=a.quantization))
    eng.start()
    for L in a.lens:
        # a token sequence of its own per length: with one shared generator the L-token prompt began
        # with the previous length's prompt, and the prefix cache served those blocks (up to round 6
        # the 2048 / 4096 rows of this probe timed 1536 / 2048 new tokens)
        ids = [100 + (j * 7919 + (0 if a.shared_prefix else 104729 * L)) % 30000 for j in range(L)]
        one(eng, f"w{L}", ids)  # eager first sight of the bucket(s)
        time.sleep(0.5)  # idle: deferred captures
        h0 = eng.snapshot().get("prefix_cache_hits", 0)
        ts = [one(eng, f"r{L}-{i}", [t + i + 1 for t in ids]) for i in range(3)]
        hits = eng.snapshot().get("prefix_cache_hits", 0) - h0  # must stay 0: every timed token is prefilled
        print(json.dumps({"model": a.model.split("/")[-1], "prompt_len": L, "chunk": a.chunk,
                          "quantization": a.quantization, "prefix_cache_hits": hits,
                          "ttft_ms": round(1e3 * min(ts), 2), "prefill_tok_s": round(L / min(ts))}), flush=True)
    eng.stop()


if __name__ == "__main__":
    main()
