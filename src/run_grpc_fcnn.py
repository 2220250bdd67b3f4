"""Reference-compatible entry point (same path and flags as /root/reference/src/run_grpc_fcnn.py).
Implementation: docker_dist_nn_amd/cli/fcnn.py."""
import os
import sys

SCRIPT_DIR = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(SCRIPT_DIR))

from docker_dist_nn_amd.cli.fcnn import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main(script_dir=SCRIPT_DIR))
