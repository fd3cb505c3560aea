"""bench.py argument checks that need no GPU: --replicas is the configs[0] (vanilla SAC) layout on one GPU only,
and the parent process refuses other configs before touching the device."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_replicas_only_for_the_vanilla_config():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--config", "sac_hopper", "--replicas", "2"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "--replicas is for --config vanilla_sac_hcheetah" in r.stderr
