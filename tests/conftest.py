import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP library + device)")
    # the HIP library is a build artefact (git-ignored): build it in-tree if absent
    libs = [os.path.join(ROOT, "modular_rl_amd", "libmrl_hip.so"), os.path.join(ROOT, "oracle", "libmrl_oracle.so")]
    if not all(os.path.exists(p) for p in libs):
        subprocess.run(["make", "-C", ROOT, "-j8", "all", "oracle"], check=True, stdout=subprocess.DEVNULL)
