"""The real-node acceptance script parses and plans every BASELINE config."""
import os
import subprocess

E2E = os.path.join(os.path.dirname(__file__), "e2e", "run_e2e.sh")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_e2e_script_syntax():
    assert subprocess.run(["bash", "-n", E2E]).returncode == 0


def test_e2e_plan_covers_configs_and_manifests_exist():
    r = subprocess.run(["bash", E2E, "--plan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    for c in range(1, 6):
        assert f"== config {c}:" in r.stdout
    applied = [l.split()[-1] for l in r.stdout.splitlines() if "kubectl apply -f" in l]
    assert len(applied) == 6
    for path in applied:
        assert os.path.exists(path), path
    assert "python3 -m mxk8s bootstrap" in r.stdout
