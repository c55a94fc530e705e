"""torchrun entrypoint, argv-compatible with the reference's main.py (main.py:178-184 (every participant trains: gradient averaging)).

See fedrec_with_pytorchdistributed_amd/cli.py for the argument contract and overrides."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from fedrec_with_pytorchdistributed_amd.cli import main_grad_avg  # noqa: E402

if __name__ == "__main__":
    sys.exit(main_grad_avg())
