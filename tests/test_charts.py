"""Helm chart rendering via tools/helmlite.py (no helm binary here)."""
import json
import os
import sys

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from helmlite import manifests, render_chart  # noqa: E402

from hipserve.gateway.ingress import rules_from_virtualservice  # noqa: E402

HF = os.path.join(ROOT, "deploy/charts/hf-models")
GG = os.path.join(ROOT, "deploy/charts/gguf-models")

# the reference vllm-models values (vllm-models/helm-chart/values.yaml:1-27), same schema
REF_HF_VALUES = {
    "models": [
        {"huggingfaceId": "leon-se/gemma-3-27b-it-FP8-Dynamic", "modelName": "gemma-3-27b-it",
         "gpuRequestCount": 2, "replicas": 1, "pvcSize": "40Gi"},
        {"huggingfaceId": "cpatonn/Qwen3-VL-30B-A3B-Instruct-AWQ-8bit", "modelName": "qwen3-vl-30b",
         "gpuRequestCount": 2, "replicas": 1, "pvcSize": "45Gi"},
    ],
    "storage": {"className": "gp2"},
}


def by_kind(docs, kind):
    return {d["metadata"]["name"]: d for d in docs if d["kind"] == kind}


def render(chart, values=None, ns="models"):
    return manifests(render_chart(chart, values or {}, namespace=ns))


def test_hf_default_render():
    docs = render(HF)
    deps = by_kind(docs, "Deployment")
    assert {"hipserve-llama-3-8b", "hipserve-mixtral-8x7b", "hipserve-api-gateway",
            "hipserve-webui"} <= set(deps)
    assert {"hipserve-llama-3-8b", "hipserve-mixtral-8x7b", "hipserve-api-gateway",
            "hipserve-webui"} <= set(by_kind(docs, "Service"))
    pvcs = by_kind(docs, "PersistentVolumeClaim")
    assert pvcs["hipserve-llama-3-8b-pvc"]["spec"]["resources"]["requests"]["storage"] == "40Gi"


def test_hf_engine_contract_matches_reference_flags():
    docs = render(HF, REF_HF_VALUES)
    d = by_kind(docs, "Deployment")["hipserve-gemma-3-27b-it"]
    c = d["spec"]["template"]["spec"]["containers"][0]
    args = c["args"]
    kv = {args[i]: args[i + 1] for i in range(len(args) - 1) if args[i].startswith("--")}
    assert kv["--model"] == "leon-se/gemma-3-27b-it-FP8-Dynamic"
    assert kv["--served-model-name"] == "gemma-3-27b-it"
    assert kv["--host"] == "0.0.0.0" and kv["--port"] == "8080"
    assert kv["--gpu-memory-utilization"] == "0.9"
    assert kv["--tensor-parallel-size"] == "2"
    assert "--trust-remote-code" in args
    assert c["resources"]["limits"]["amd.com/gpu"] == 2
    assert c["resources"]["requests"]["amd.com/gpu"] == 2
    for p in ("startupProbe", "readinessProbe", "livenessProbe"):
        assert c[p]["httpGet"]["path"] == "/health"
    mounts = {m["name"]: m["mountPath"] for m in c["volumeMounts"]}
    assert mounts == {"model-cache": "/root/.cache/huggingface", "dshm": "/dev/shm"}
    vols = {v["name"]: v for v in d["spec"]["template"]["spec"]["volumes"]}
    assert vols["dshm"]["emptyDir"]["medium"] == "Memory"
    assert vols["model-cache"]["persistentVolumeClaim"]["claimName"] == "hipserve-gemma-3-27b-it-pvc"
    env = {e["name"]: e for e in c["env"]}
    tok = env["HUGGING_FACE_HUB_TOKEN"]["valueFrom"]["secretKeyRef"]
    assert tok["name"] == "huggingface-token" and tok["key"] == "token" and tok["optional"] is True
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"]["value"] == "0"
    tol = d["spec"]["template"]["spec"]["tolerations"]
    assert tol[0]["key"] == "amd.com/gpu"
    ann = d["spec"]["template"]["metadata"]["annotations"]
    assert ann["prometheus.io/scrape"] == "true"
    pvc = by_kind(docs, "PersistentVolumeClaim")["hipserve-gemma-3-27b-it-pvc"]
    assert pvc["spec"]["storageClassName"] == "gp2"
    assert pvc["spec"]["accessModes"] == ["ReadWriteOnce"]


def test_hf_replicas_get_rwx_and_extra_args():
    vals = {"models": [{"huggingfaceId": "m/x", "modelName": "x", "gpuRequestCount": 1, "replicas": 3,
                        "pvcSize": "10Gi", "maxModelLen": 4096, "loadFormat": "dummy",
                        "engineArgs": ["--enforce-eager"]}]}
    docs = render(HF, vals)
    pvc = by_kind(docs, "PersistentVolumeClaim")["hipserve-x-pvc"]
    assert pvc["spec"]["accessModes"] == ["ReadWriteMany"]
    d = by_kind(docs, "Deployment")["hipserve-x"]
    assert d["spec"]["replicas"] == 3
    args = d["spec"]["template"]["spec"]["containers"][0]["args"]
    assert args[args.index("--max-model-len") + 1] == "4096"
    assert args[args.index("--load-format") + 1] == "dummy"
    assert "--enforce-eager" in args


def test_hf_virtualservice_order_and_ingress_emulation():
    docs = render(HF)
    vs = by_kind(docs, "VirtualService")["hipserve-virtual-service"]
    http = vs["spec"]["http"]
    assert http[0]["match"][0]["uri"] == {"exact": "/v1/models"}
    assert http[1]["match"][0]["uri"] == {"prefix": "/v1/"}
    assert http[2]["match"][0]["uri"] == {"prefix": "/health"}
    assert http[3]["match"][0]["uri"] == {"prefix": "/"}
    assert http[3]["route"][0]["destination"]["host"] == "hipserve-webui"
    rules = rules_from_virtualservice(docs)
    hit = lambda p: next(r.host for r in rules if r.hit(p))  # noqa: E731
    assert hit("/v1/models") == hit("/v1/chat/completions") == hit("/health") == "hipserve-api-gateway"
    assert hit("/") == hit("/chat/x") == "hipserve-webui"
    gw = by_kind(docs, "Gateway")["hipserve-gateway"]
    assert gw["spec"]["servers"][0]["port"]["number"] == 80


def test_hf_nginx_router_fixed_config():
    docs = render(HF, {"apiGateway": {"kind": "nginx"}})
    cm = by_kind(docs, "ConfigMap")["hipserve-api-gateway-config"]
    conf = cm["data"]["nginx.conf"]
    for needle in ("proxy_buffering off;", "proxy_http_version 1.1;", "client_max_body_size 0;",
                   "get_body_file", "upstream hipserve-llama-3-8b", "upstream hipserve-mixtral-8x7b",
                   'set $upstream "hipserve-llama-3-8b"', "location = /v1/models", "location = /health",
                   "proxy_read_timeout 3600s;", "keepalive"):
        assert needle in conf, needle
    assert conf.count("{") == conf.count("}")


def test_hf_hipserve_router_default():
    docs = render(HF, {}, ns="prod")
    cm = by_kind(docs, "ConfigMap")["hipserve-api-gateway-config"]
    backends = json.loads(cm["data"]["backends.json"])
    assert [b["name"] for b in backends] == ["llama-3-8b", "mixtral-8x7b"]
    assert backends[0]["url"] == "http://hipserve-llama-3-8b.prod.svc.cluster.local:8080"
    d = by_kind(docs, "Deployment")["hipserve-api-gateway"]
    cmd = d["spec"]["template"]["spec"]["containers"][0]["command"]
    assert cmd[:4] == ["python3", "-m", "hipserve.gateway", "router"]


def test_empty_models_fails_loudly():
    with pytest.raises(ValueError, match="at least one model"):
        render_chart(HF, {"models": []})
    with pytest.raises(ValueError, match="at least one model"):
        render_chart(GG, {"models": []})


def test_name_prefix_and_shared_gateway():
    docs = render(HF, {"namePrefix": "team-a", "istio": {"createGateway": False, "gatewayName": "shared"}})
    assert "Gateway" not in {d["kind"] for d in docs}
    vs = by_kind(docs, "VirtualService")["team-a-virtual-service"]
    assert vs["spec"]["gateways"] == ["shared"]
    assert "team-a-llama-3-8b" in by_kind(docs, "Deployment")


def test_gguf_render_and_llama_server_contract():
    docs = render(GG, ns="default")
    deps = by_kind(docs, "Deployment")
    d = deps["gguf-models-tinyllama"]
    c = d["spec"]["template"]["spec"]["containers"][0]
    assert c["command"] == ["hipserve-llama-server"]
    a = c["args"]
    assert a[a.index("--model") + 1] == "/mnt/models/tinyllama-1.1b-chat-v1.0.Q4_0.gguf"
    assert a[a.index("--alias") + 1] == "tinyllama"
    assert a[a.index("--host") + 1] == "0.0.0.0" and a[a.index("--port") + 1] == "8080"
    assert c["resources"]["limits"]["amd.com/gpu"] == 1
    assert all(p in c for p in ("readinessProbe", "livenessProbe", "startupProbe"))
    vols = {v["name"]: v for v in d["spec"]["template"]["spec"]["volumes"]}
    assert vols["models"]["hostPath"]["path"] == "/mnt/models"
    cm = by_kind(docs, "ConfigMap")["gguf-models-api-gateway-config"]
    b = json.loads(cm["data"]["backends.json"])
    assert b[0] == {"name": "tinyllama",
                    "url": "http://gguf-models-tinyllama.default.svc.cluster.local:8080"}
    assert deps["gguf-models-api-gateway"]["spec"]["replicas"] == 2
    vs = by_kind(docs, "VirtualService")["gguf-models-virtual-service"]
    assert vs["spec"]["http"][0]["match"][0]["uri"] == {"prefix": "/v1"}
    assert vs["spec"]["http"][0]["route"][0]["destination"]["host"] == \
        "gguf-models-api-gateway.default.svc.cluster.local"
    webui = deps["gguf-models-webui"]["spec"]["template"]["spec"]["containers"][0]
    env = {e["name"]: e["value"] for e in webui["env"]}
    assert env["OPENAI_API_BASE_URLS"] == "http://gguf-models-api-gateway:8080/v1"


def test_gguf_webui_without_persistence_has_no_dangling_volume():
    docs = render(GG, {"webui": {"persistence": {"enabled": False}}})
    assert "PersistentVolumeClaim" not in {d["kind"] for d in docs}
    spec = by_kind(docs, "Deployment")["gguf-models-webui"]["spec"]["template"]["spec"]
    assert "volumes" not in spec and "volumeMounts" not in spec["containers"][0]


def test_gguf_fullname_from_release():
    docs = manifests(render_chart(GG, {"fullnameOverride": ""}, release="prod"))
    assert "prod-gguf-models-tinyllama" in by_kind(docs, "Deployment")


@pytest.mark.parametrize("app", sorted(os.listdir(os.path.join(ROOT, "deploy/argocd"))))
def test_argocd_applications_render(app):
    with open(os.path.join(ROOT, "deploy/argocd", app)) as f:
        a = yaml.safe_load(f)
    assert a["kind"] == "Application" and a["apiVersion"] == "argoproj.io/v1alpha1"
    src = a["spec"]["source"]
    chart = os.path.join(ROOT, src["path"])
    assert os.path.exists(os.path.join(chart, "Chart.yaml"))
    vals = yaml.safe_load(src["helm"]["values"])
    docs = manifests(render_chart(chart, vals, namespace=a["spec"]["destination"]["namespace"]))
    assert any(d["kind"] == "Deployment" for d in docs)
    sp = a["spec"]["syncPolicy"]["automated"]
    assert sp["prune"] and sp["selfHeal"]


def test_hf_engine_log_format_env():
    """engine.logFormat reaches the pod as HIPSERVE_LOG_FORMAT (text by default)."""
    def env_of(values):
        d = by_kind(render(HF, values), "Deployment")["hipserve-llama-3-8b"]
        env = d["spec"]["template"]["spec"]["containers"][0]["env"]
        return {e["name"]: e.get("value") for e in env}

    assert env_of({})["HIPSERVE_LOG_FORMAT"] == "text"
    assert env_of({"engine": {"logFormat": "json"}})["HIPSERVE_LOG_FORMAT"] == "json"


def _env(dep):
    return {e["name"]: e.get("value") for e in dep["spec"]["template"]["spec"]["containers"][0]["env"]}


def test_tune_cache_persisted_on_model_volume():
    """the start-up tuning tables live on storage that outlives the
    pod (the reference keeps its engine cache on the model PVC,
    vllm-models/helm-chart/templates/model-deployments.yaml:45-47,71-74)."""
    d = by_kind(render(HF), "Deployment")["hipserve-llama-3-8b"]
    path = _env(d)["HIPSERVE_TUNE_CACHE"]
    c = d["spec"]["template"]["spec"]["containers"][0]
    mounts = {m["name"]: m["mountPath"] for m in c["volumeMounts"]}
    assert path.startswith(mounts["model-cache"] + "/")  # on the per-model PVC
    vols = {v["name"]: v for v in d["spec"]["template"]["spec"]["volumes"]}
    assert "persistentVolumeClaim" in vols["model-cache"]
    d = by_kind(render(HF, {"engine": {"tuneCacheDir": "0"}}), "Deployment")["hipserve-llama-3-8b"]
    assert _env(d)["HIPSERVE_TUNE_CACHE"] == "0"

    g = by_kind(render(GG), "Deployment")["gguf-models-tinyllama"]
    spec = g["spec"]["template"]["spec"]
    mounts = {m["name"]: m for m in spec["containers"][0]["volumeMounts"]}
    vols = {v["name"]: v for v in spec["volumes"]}
    assert _env(g)["HIPSERVE_TUNE_CACHE"] == mounts["tune-cache"]["mountPath"]
    assert not mounts["tune-cache"].get("readOnly")
    assert vols["tune-cache"]["hostPath"]["type"] == "DirectoryOrCreate"
    g = by_kind(render(GG, {"tuneCache": {"hostPath": ""}}), "Deployment")["gguf-models-tinyllama"]
    assert "emptyDir" in {v["name"]: v for v in g["spec"]["template"]["spec"]["volumes"]}["tune-cache"]
