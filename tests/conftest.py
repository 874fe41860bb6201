import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger parity cases")


@pytest.fixture(scope="session")
def match_test_db_json():
    import json
    with open(os.path.join(GOLDEN, "match_test_db.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def refdb(match_test_db_json):
    from oracle.match_ref import RefDB
    return RefDB.from_json(match_test_db_json)
