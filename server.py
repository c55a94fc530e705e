"""torchrun entrypoint, argv-compatible with the reference's server.py (server.py:108-114).

See fedrec_with_pytorchdistributed_amd/cli.py for the argument contract and overrides."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from fedrec_with_pytorchdistributed_amd.cli import main_server  # noqa: E402

if __name__ == "__main__":
    sys.exit(main_server())
