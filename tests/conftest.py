import importlib.util
import os
import sys

import pytest

# torch first: it ships its own HIP runtime, and the process must use ONE copy of libamdhip64. When
# torch is imported after the library has already loaded the system runtime, torch's device init
# fails ("No HIP GPUs are available"), so the GPU tests that hand torch buffers to the library
# (shard gather) would depend on collection order.
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ray-tracing-project_amd")
SCENES = os.path.join(ROOT, "scenes")
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


rtamd = _load("rtamd", os.path.join(PKG, "rtamd.py"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the gfx950 kernels)")


# Parity summaries the full-frame GPU tests add (printed at the end of the run, so the driver's record of
# the test tail carries the measured per-frame error, not only a pass count)
PARITY_REPORT = []


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if PARITY_REPORT:
        terminalreporter.write_sep("-", "full-frame parity vs the CPU oracle")
        for line in PARITY_REPORT:
            terminalreporter.write_line(line)


@pytest.fixture(scope="session")
def rt():
    rtamd.lib()
    return rtamd


@pytest.fixture(scope="session")
def orc():
    import oracle
    oracle.lib()
    return oracle


def scene_path(name):
    return os.path.join(SCENES, name)
