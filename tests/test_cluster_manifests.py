"""GPU-node provisioning as applied YAML (deploy/cluster/mi355x-node/, the MI355X
counterpart of the reference's eksctl ClusterConfig,
vllm-models/eks-cluster-config.yaml:1-59): every document parses, and the node
labels / taint / storage class agree with what the charts, the device plugin and
the Argo CD Applications select on."""
import os

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = os.path.join(ROOT, "deploy", "cluster", "mi355x-node")


def _docs(path):
    with open(path) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def _values(chart):
    with open(os.path.join(ROOT, "deploy", "charts", chart, "values.yaml")) as f:
        return yaml.safe_load(f)


def test_manifests_parse_and_kustomization_resolves():
    kust = _docs(os.path.join(NODE, "kustomization.yaml"))[0]
    assert kust["kind"] == "Kustomization"
    for r in kust["resources"]:
        p = os.path.normpath(os.path.join(NODE, r))
        assert os.path.exists(p), r
        assert _docs(p)
    for f in os.listdir(NODE):
        if f.endswith(".yaml"):
            assert _docs(os.path.join(NODE, f)), f


def test_kubeadm_node_matches_chart_scheduling():
    docs = {d["kind"]: d for d in _docs(os.path.join(NODE, "kubeadm-config.yaml"))}
    init = docs["InitConfiguration"]["nodeRegistration"]
    taints = {(t["key"], t["effect"]) for t in init["taints"]}
    labels = dict(kv.split("=") for a in init["kubeletExtraArgs"] if a["name"] == "node-labels"
                  for kv in a["value"].split(","))
    tol = {(t["key"], t["effect"]) for t in _values("hf-models")["gpu"]["tolerations"]}
    assert taints <= tol  # model pods tolerate every taint the node carries
    plugin = _docs(os.path.join(ROOT, "deploy", "cluster", "amd-gpu-device-plugin.yaml"))[0]
    sel = plugin["spec"]["template"]["spec"]["nodeSelector"]
    assert all(labels.get(k) == v for k, v in sel.items())  # the device plugin lands on the node
    ptol = {(t["key"], t["effect"]) for t in plugin["spec"]["template"]["spec"]["tolerations"] if "effect" in t}
    assert taints <= ptol
    assert labels["amd.com/gpu.arch"] == "gfx950"
    kub = docs["KubeletConfiguration"]
    assert kub["cpuManagerPolicy"] == "static" and kub["topologyManagerPolicy"] in ("best-effort", "restricted")


def test_k3s_config_equivalent():
    k3s = _docs(os.path.join(NODE, "k3s-config.yaml"))[0]
    assert "node-type=gpu" in k3s["node-label"]
    assert "amd.com/gpu=true:NoSchedule" in k3s["node-taint"]
    assert "traefik" in k3s["disable"]


def test_storage_class_used_by_gpu_applications():
    sc = [d for d in _docs(os.path.join(NODE, "storageclass-weights.yaml")) if d["kind"] == "StorageClass"][0]
    name = sc["metadata"]["name"]
    assert sc["volumeBindingMode"] == "WaitForFirstConsumer" and sc["reclaimPolicy"] == "Retain"
    for app in ("hf-models.yaml", "llama-3-70b-tp8.yaml"):
        a = _docs(os.path.join(ROOT, "deploy", "argocd", app))[0]
        vals = yaml.safe_load(a["spec"]["source"]["helm"]["values"])
        assert vals["storage"]["className"] == name, app
    ns = _docs(os.path.join(NODE, "namespaces.yaml"))
    q = [d for d in ns if d["kind"] == "ResourceQuota"][0]
    assert q["spec"]["hard"]["requests.amd.com/gpu"] == "8"
