import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "sparkey-java_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def native():
    """The HIP library (built in-tree if missing)."""
    import build as sk_build  # sparkey-java_amd/build.py
    sk_build.build()
    from sparkey import _native
    return _native


@pytest.fixture
def switch(native):
    """switch(name=value, ...): sets the library's test switches (sparkey_debug_set) for this test;
    every switch it touched is unset again at teardown."""
    touched = set()

    def set_(**kv):
        for k, v in kv.items():
            native.debug_set(k, v)
            touched.add(k)

    yield set_
    for k in touched:
        native.debug_set(k, None)
