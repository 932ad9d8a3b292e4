"""World-N rehearsal of the training loop (hzamd.trainer.Trainer, BASELINE
config 5) for tests/test_multirank_gpu.py: launched by torch.distributed.run
with gloo, every rank on cuda:0 (a one-GPU box), or with RCCL at one rank
(HZ_DIST_BACKEND=nccl).  Each rank writes what it
ended with: model and best-model weights, replay buffer, history."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "harmonies-alphazero_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(out, folder):
    from hzamd.manager import ModelManager
    from hzamd.trainer import Trainer
    from test_manager_cpu import MODEL_CFG
    from test_trainer_gpu import EVAL, MCTS, TRAIN
    torch.cuda.set_device(0)
    if os.environ.get("HZ_DETERMINISTIC", "1") == "1":
        # training in a fixed summation order (PyTorch's own conv kernels
        # instead of MIOpen's, whose backward reductions vary run to run), so
        # two runs of the loop over different backends end with the same
        # weights and the broadcast can be compared bit for bit
        torch.backends.cudnn.enabled = False
        torch.use_deterministic_algorithms(True)  # an op without a deterministic form raises here
    backend = os.environ.get("HZ_DIST_BACKEND", "gloo")  # "nccl" (RCCL): one rank only on a one-GPU box
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend)
    rank = dist.get_rank()
    torch.manual_seed(100 + rank)  # ranks start from different weights: the broadcast must fix that
    cfg = {"num_iterations": 2, "num_games_per_iter": 6, "epochs_per_iter": 1, "replay_buffer_size": 1000,
           "checkpoint_folder": os.path.join(folder, "ck"), "replay_buffer_folder": os.path.join(folder, "buf"),
           "replay_buffer_filename": "rb.pkl", "eval_frequency": 2, "eval_episodes": 5,
           "eval_win_rate_threshold": 0.0, "best_model_filename": "best.pth.tar"}
    mm = ModelManager(MODEL_CFG, TRAIN)
    tr = Trainer(mm, MCTS, cfg, TRAIN, eval_mcts_config=EVAL, seed_base=7, log=lambda *_: None)
    hist = tr.run_training_loop()
    flat = lambda m: torch.cat([t.detach().reshape(-1).double().cpu() for t in m.state_dict().values()])  # noqa
    torch.save({"model": flat(tr.model_manager.model), "best": flat(tr.best_model_manager.model),
                "buffer": tr.replay_buffer.records().cpu(),
                "evals": [h["evaluation"] for h in hist], "examples": [h["self_play"]["examples"] for h in hist],
                "world": dist.get_world_size(), "backend": dist.get_backend()}, f"{out}.rank{rank}.pt")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
