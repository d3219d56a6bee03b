"""Config loader: schema defaults, YAML, env overrides with __ nesting, priority, validators."""
import json

import pytest
from pydantic import ValidationError

from vgate.config import VGateConfig, env_overrides, get_config, load_config, reset_config


def test_defaults_match_reference_schema(clean_env):
    c = VGateConfig()
    assert c.version == "0.3.2" and c.role == "gateway"
    assert (c.server.host, c.server.port) == ("0.0.0.0", 8000)
    assert c.worker.endpoints == [] and c.worker.discovery.dns_name is None
    assert (c.worker.timeout_seconds, c.worker.connect_timeout_seconds) == (120.0, 5.0)
    assert (c.worker.failure_threshold, c.worker.success_threshold) == (2, 2)
    assert c.model.model_id == "Qwen/Qwen2.5-1.5B-Instruct-AWQ" and c.model.quantization == "awq"
    assert c.model.max_model_len == 2048 and c.model.gpu_memory_utilization == 0.7
    assert (c.batch.max_batch_size, c.batch.max_wait_time_ms) == (8, 50.0)
    assert (c.cache.enabled, c.cache.maxsize) == (True, 1000)
    assert (c.inference.temperature, c.inference.top_p, c.inference.max_tokens) == (0.7, 0.9, 256)
    assert c.security.enabled is False and c.security.exempt_paths == ["/health", "/metrics"]
    assert c.security.rate_limiting.window_seconds == 60
    assert len(c.benchmark.prompts) == 3
    assert c.tracing.otlp_endpoint == "http://localhost:4317"


def test_yaml_then_env_priority(tmp_path, clean_env):
    p = tmp_path / "c.yaml"
    p.write_text("server:\n  port: 9000\n  host: 127.0.0.1\nmodel:\n  model_id: foo\n  max_model_len: 4096\n")
    c = load_config(p)
    assert c.server.port == 9000 and c.model.model_id == "foo"
    clean_env.setenv("VGATE_SERVER__PORT", "9100")
    c = load_config(p)
    assert c.server.port == 9100  # env beats yaml
    assert c.server.host == "127.0.0.1"  # sibling yaml key survives (deep merge)
    assert c.model.max_model_len == 4096


def test_init_beats_env(clean_env):
    clean_env.setenv("VGATE_SERVER__PORT", "9100")
    assert VGateConfig(server={"port": 7000}).server.port == 7000


def test_env_json_values(clean_env):
    clean_env.setenv("VGATE_WORKER__ENDPOINTS", json.dumps(["http://w1:8000/", "http://w2:8000"]))
    clean_env.setenv("VGATE_SECURITY__API_KEYS", json.dumps([{"key": "k1", "name": "a", "rate_limit": 5}]))
    clean_env.setenv("VGATE_SECURITY__ENABLED", "true")
    clean_env.setenv("VGATE_CACHE__MAXSIZE", "42")
    c = VGateConfig()
    assert c.worker.endpoints == ["http://w1:8000", "http://w2:8000"]  # trailing slash stripped
    assert c.security.api_keys[0].rate_limit == 5 and c.security.enabled is True
    assert c.cache.maxsize == 42


def test_non_schema_env_vars_ignored(clean_env):
    clean_env.setenv("VGATE_DRY_RUN", "true")
    clean_env.setenv("VGATE_CONFIG_PATH", "/nope")
    assert "dry_run" not in env_overrides()
    VGateConfig()


@pytest.mark.parametrize("kw", [{"role": "boss"}, {"model": {"engine_type": "tgi"}},
                                {"worker": {"endpoints": ["w1:8000"]}},
                                {"worker": {"discovery": {"scheme": "ftp"}}},
                                {"model": {"quantization": "gptq"}}])
def test_validators(kw, clean_env):
    with pytest.raises(ValidationError):
        VGateConfig(**kw)


def test_engine_type_aliases_accepted(clean_env):
    for t in ("native", "vllm", "sglang"):
        assert VGateConfig(model={"engine_type": t}).model.engine_type == t


def test_get_config_singleton_and_path(tmp_path, clean_env, monkeypatch):
    p = tmp_path / "x.yaml"
    p.write_text("version: '9.9'\n")
    clean_env.setenv("VGATE_CONFIG_PATH", str(p))
    reset_config()
    assert get_config().version == "9.9"
    assert get_config() is get_config()
    reset_config()
    clean_env.delenv("VGATE_CONFIG_PATH")
    monkeypatch.chdir(tmp_path)
    assert get_config().version == "0.3.2"


def test_missing_yaml_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        load_config(tmp_path / "missing.yaml")


def test_repo_config_yaml_loads(clean_env):
    from pathlib import Path
    c = load_config(Path(__file__).resolve().parents[1] / "config.yaml")
    assert c.model.engine_type == "native"
