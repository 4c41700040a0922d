import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "raytracer-server_amd"))

SCENES = os.path.join(REPO, "scenes")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def scene_path(name):
    return os.path.join(SCENES, f"{name}.toml")


@pytest.fixture(scope="session")
def oracle():
    import oracle_bind

    oracle_bind.lib()
    return oracle_bind


@pytest.fixture(scope="session")
def oracle_scenes(oracle):
    return {n: oracle.OracleScene(scene_path(n)) for n in ("cornell_box", "cubes", "flying_unicorn")}


@pytest.fixture(scope="session")
def rt():
    import rt_amd

    return rt_amd


@pytest.fixture(scope="session")
def gpu_scenes(rt):
    if rt.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests need an MI355X")
    return {n: rt.Scene.from_toml(scene_path(n)) for n in ("cornell_box", "cubes", "flying_unicorn")}
