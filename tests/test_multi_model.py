"""Multi-model serving path (BASELINE config 5) on CPU: two engine processes
(Llama and Mixtral architectures) behind the model-name router and the ingress
emulator; per-model and concurrent phases must all complete."""
import json

from hipserve.bench import multi_model


def test_multi_model_bench_cpu(tmp_path):
    out = tmp_path / "mm.jsonl"
    multi_model.main(["--models", "tiny-llama,tiny-mixtral", "--device", "cpu", "--kv-blocks", "256",
                      "--concurrency", "2", "--input-len", "16", "--output-len", "4", "--waves", "1",
                      "--warmup", "0", "--out", str(out)])
    lines = [json.loads(x) for x in out.read_text().splitlines()]
    assert [ln["phase"] for ln in lines] == ["tiny-llama alone", "tiny-mixtral alone", "all models concurrently"]
    both = lines[-1]["models"]
    assert set(both) == {"tiny-llama", "tiny-mixtral"}
    for m in both.values():
        assert m["requests"] == 2 and m["output_tok_per_s"] > 0 and m["p50_ttft_ms"] is not None
