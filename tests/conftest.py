import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmythgpu.so)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def oracle_evm():
    from oracle.evm_ref import OracleEVM
    return OracleEVM


@pytest.fixture(autouse=True)
def _fresh_function_managers():
    """The keccak and exponent managers are process globals (as in the
    reference): every test starts from empty registries, so a symbolic run in
    one test cannot leave keccak inputs that make another test's empty
    constraint set undecidable.  reset() keeps the keccak interval counter, as
    the reference's does."""
    from mythril_amd.smt.exponent_manager import exponent_function_manager
    from mythril_amd.smt.keccak_manager import keccak_function_manager
    keccak_function_manager.reset()
    exponent_function_manager.reset()
    yield
