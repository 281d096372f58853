"""Config schema (mxk8s/config.py): chart values, values.schema.json and the
bootstrap settings stay in agreement; bad values are rejected with paths."""
import json
import os
import subprocess
import sys

import pytest
import yaml

from mxk8s import config
from mxk8s.bootstrap import hostfiles as hf
from mxk8s.bootstrap import phases
from mxk8s.chart import render

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chart_defaults_validate_and_schema_file_is_current():
    with open(os.path.join(config.CHART_DIR, "values.yaml")) as f:
        values = yaml.safe_load(f)
    assert config.validate_values(values) == []
    with open(os.path.join(config.CHART_DIR, "values.schema.json")) as f:
        assert json.load(f) == config.values_schema_document(), \
            "run `python -m mxk8s.config write` after changing mxk8s/config.py"
    # every key of values.yaml is described by the schema and vice versa
    def keys(d, spec, pre=""):
        for k, v in d.items():
            assert k in spec, f"{pre}{k} missing from config.VALUES"
            if isinstance(spec[k], dict):
                keys(v, spec[k], f"{pre}{k}.")
        for k in spec:
            assert k in d, f"{pre}{k} in config.VALUES but not in values.yaml"
    keys(values, config.VALUES)


@pytest.mark.parametrize("sets,needle", [
    (["validator.gpus=9"], "validator.gpus: 9 > maximum 8"),
    (["exporter.port=0"], "exporter.port: 0 < minimum 1"),
    (["validator.tests={gemm,bogus}"], "validator.tests[1]"),
    (["validator.rccl.ops={allreduce,broadcast}"], "validator.rccl.ops[1]"),
    (["devicePlugin.healtInterval=3"], "devicePlugin.healtInterval: unknown key"),
    (["resourceName=gpu"], "resourceName"),
    (["driver.enabled=true"], "not supported"),
    (["validator.rccl.minBytes=1024", "validator.rccl.maxBytes=8"], "minBytes > maxBytes"),
])
def test_bad_values_rejected(sets, needle):
    values = render.load_values(render.CHART_DIR, [], sets)
    errs = config.validate_values(values)
    assert any(needle in e for e in errs), errs


def test_render_cli_reports_schema_errors():
    r = subprocess.run([sys.executable, "-m", "mxk8s", "render", "--set", "validator.gpus=0"],
                       capture_output=True, text=True, env={**os.environ, "PYTHONPATH": REPO})
    assert r.returncode == 1 and "validator.gpus: 0 < minimum 1" in r.stderr


def test_bootstrap_precedence(tmp_path):
    toml = tmp_path / "mxk8s.toml"
    toml.write_text('[bootstrap]\nnode_name = "from-file"\npod_cidr = "10.50.0.0/16"\n'
                    'upgrade = true\n')
    cfg = config.load_bootstrap(str(toml), env={})
    assert (cfg["node_name"], cfg["pod_cidr"], cfg["upgrade"]) == ("from-file", "10.50.0.0/16", True)
    cfg = config.load_bootstrap(str(toml), env={"MXK8S_NODE_NAME": "from-env",
                                                "MXK8S_UPGRADE": "no"})
    assert (cfg["node_name"], cfg["upgrade"]) == ("from-env", False)
    cfg = config.load_bootstrap(str(toml), env={"MXK8S_NODE_NAME": "from-env"},
                                overrides={"node_name": "from-flag", "root": None})
    assert cfg["node_name"] == "from-flag" and cfg["root"] == "/"
    assert config.load_bootstrap(None, env={})["pod_cidr"] == hf.POD_CIDR


@pytest.mark.parametrize("text,err", [
    ('[bootstrap]\npod_cidr = "10.244.0.0/33"\n', "pod_cidr"),
    ('[bootstrap]\nkubernetes_version = "1.34"\n', "kubernetes_version"),
    ('[bootstrap]\nnode_nam = "x"\n', "unknown bootstrap setting"),
    ('[bootstrap]\nupgrade = "maybe"\n', "not a boolean"),
])
def test_bootstrap_config_errors(tmp_path, text, err):
    p = tmp_path / "bad.toml"
    p.write_text(text)
    with pytest.raises(ValueError, match=err):
        config.load_bootstrap(str(p), env={})


def test_custom_pod_cidr_reaches_kubeadm_and_flannel(tmp_path):
    ctx = phases.Context(root=str(tmp_path), dry_run=True, pod_cidr="10.50.0.0/16",
                         kubernetes_version="v1.34.2")
    ctx.out = lambda s: None
    phases.phase_cluster(ctx)
    kc = list(yaml.safe_load_all(open(tmp_path / "etc/mxk8s/kubeadm-config.yaml")))
    assert kc[1]["networking"]["podSubnet"] == "10.50.0.0/16"
    assert kc[1]["kubernetesVersion"] == "v1.34.2"
    fl = open(tmp_path / "etc/mxk8s/kube-flannel.yaml").read()
    assert '"Network": "10.50.0.0/16"' in fl and '"Network": "10.244.0.0/16"' not in fl
    assert hf.k8s_minor("v1.34.2") == "v1.34"
