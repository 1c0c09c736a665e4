"""Distributed MNIST CNN trainer -- entry point with the reference's defaults for this role
(/root/reference/mnist_python_m.py: task_index=0, job_name="ps"; the three reference scripts are
one program with different flag defaults).

    python mnist_python_m.py --ps_hosts=127.0.0.1:2222 --worker_hosts=127.0.0.1:2223,127.0.0.1:2224 \
        [--job_name=... --task_index=... --num_gpus=1 --sync_replicas=True --train_steps=4]

Sync mode = RCCL (GPU) / Gloo (CPU) all-reduce DP with SyncReplicasOptimizer semantics; async mode
= Hogwild parameter server. See tensorflow_distributed_amd/training/dist_main.py.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from tensorflow_distributed_amd.training.dist_main import run_script  # noqa: E402

if __name__ == "__main__":
    sys.exit(run_script(task_index_default=0, job_name_default="ps"))
