"""The reference's training loop (trainer.py Trainer, main.py) on the batched
GPU engine (BASELINE config 5).

Same phases and configuration keys as trainer.Trainer:
  execute_self_play_phase  trainer.py:62-134   num_games_per_iter games per
                           rank played at once (hzamd.selfplay.SelfPlay) with
                           the best model; records all-gathered over RCCL
                           into every rank's device replay buffer
  execute_training_phase   trainer.py:136-193  rank 0 trains from the device
                           records (hzamd.train), then broadcasts the weights
  evaluate_model           trainer.py:293-375  batched arena (hzamd.arena):
                           candidate vs best with the eval search config,
                           promotion above eval_win_rate_threshold
  run_training_loop        trainer.py:195-260  resume from
                           latest_candidate.pth.tar, iterate, checkpoint,
                           save the buffer, evaluate every eval_frequency
Checkpoints use the reference format (hzamd.manager); the buffer is saved
in the compact format (hzamd.buffer_io), with the reference pickle written
alongside when self_play_config["export_reference_pickle"] is set.
"""
import copy
import os
import time
from pathlib import Path

import torch
import torch.distributed as dist

from . import arena
from . import buffer_io
from . import distributed as hd
from .manager import ModelManager
from .mcts import BatchedPredictor
from .selfplay import SelfPlay
from .train import featurize, training_phase


def _dist():
    return dist.is_available() and dist.is_initialized()


class Trainer:
    def __init__(self, model_manager, mcts_config, self_play_config, training_config, eval_mcts_config=None,
                 seed_base=0, log=print):
        self.model_manager = model_manager
        self.mcts_config = mcts_config
        self.self_play_config = self_play_config
        self.training_config = training_config
        self.eval_mcts_config = dict(arena.MCTS_EVAL, **(eval_mcts_config or {}))
        self.seed_base = int(seed_base)
        self.log = log
        self.rank = dist.get_rank() if _dist() else 0
        self.world = dist.get_world_size() if _dist() else 1
        self.device = model_manager.device
        self.replay_buffer = hd.ReplayBuffer(self_play_config["replay_buffer_size"], self.device)
        path = self._buffer_path()
        if os.path.exists(path):
            rec, _ = buffer_io.load_compact(path, self.device)
            self.replay_buffer.extend(rec)
        self.best_model_filename = self_play_config.get("best_model_filename", "best_model.pth.tar")
        self.iteration = 0
        self.start_iteration = 0
        self._initialize_best_model()

    # -- helpers -------------------------------------------------------------
    def _buffer_path(self):
        c = self.self_play_config
        name = os.path.splitext(c.get("replay_buffer_filename", "replay_buffer.pkl"))[0] + ".hz.npz"
        return os.path.join(c.get("replay_buffer_folder", "."), name)

    def _initialize_best_model(self):
        """trainer.py:262-290: load the best checkpoint, or save the current
        model as the initial best.  Under torch.distributed only rank 0
        decides (does a loadable best checkpoint exist?); every rank then
        takes the same, unconditional barrier before the others load."""
        folder = self.self_play_config["checkpoint_folder"]
        self.best_model_manager = ModelManager(copy.deepcopy(self.model_manager.model_config),
                                               copy.deepcopy(self.model_manager.training_config))
        loaded = False
        if self.rank == 0:
            loaded, _ = self.best_model_manager.load_checkpoint(folder=folder, filename=self.best_model_filename)
            if not loaded:
                self.model_manager.save_checkpoint(folder=folder, filename=self.best_model_filename)
        if _dist():
            dist.barrier()  # the file rank 0 may just have written is complete
        if self.rank != 0 or not loaded:
            self.best_model_manager.load_checkpoint(folder=folder, filename=self.best_model_filename)

    # -- phases --------------------------------------------------------------
    def execute_self_play_phase(self, data_generating_manager):
        t0 = time.time()
        n = int(self.self_play_config["num_games_per_iter"])
        base = self.seed_base + (self.iteration * self.world + self.rank) * n
        sp = SelfPlay(n, BatchedPredictor(data_generating_manager.model), self.mcts_config, seed_base=base,
                      device=self.device)
        packed, rec = sp.iteration(self.replay_buffer)
        self.last_self_play = {"examples": int(packed.shape[0]), "games": n * self.world,
                               "plies": rec["plies"], "seconds": time.time() - t0}
        self.log(f"self-play: {self.last_self_play['games']} games, {self.last_self_play['examples']} examples, "
                 f"buffer {len(self.replay_buffer)}/{self.replay_buffer.capacity}, "
                 f"{self.last_self_play['seconds']:.2f}s")
        return self.last_self_play

    def execute_training_phase(self):
        res = None
        if self.rank == 0:
            res = training_phase(self.model_manager, featurize(self.replay_buffer.records()),
                                 self.self_play_config["epochs_per_iter"], self.training_config["batch_size"])
        if _dist():
            hd.broadcast_weights(self.model_manager.model, src=0)
        self.last_training = res
        if res is None:
            self.log("training: not enough data in buffer yet")
        else:
            self.log(f"training: avg loss {res['loss']:.4f} (policy {res['policy_loss']:.4f}, "
                     f"value {res['value_loss']:.4f}) over {res['batches']} batches")
        return res

    def evaluate_model(self):
        """trainer.py:293-375: the eval_episodes games are sharded over the
        ranks and their counts all-reduced (hzamd.arena.evaluate_model), so
        the promotion decision is the same on every rank; the barrier before
        the reload is unconditional on all ranks whenever it is taken."""
        c = self.self_play_config
        res = arena.evaluate_model(BatchedPredictor(self.model_manager.model),
                                   BatchedPredictor(self.best_model_manager.model),
                                   n_games=c["eval_episodes"], threshold=c["eval_win_rate_threshold"],
                                   mcts_config=self.eval_mcts_config,
                                   seed_base=self.seed_base + 10**9 + self.iteration * c["eval_episodes"],
                                   device=self.device)
        if res["passed"]:
            folder = c["checkpoint_folder"]
            if self.rank == 0:
                self.model_manager.save_checkpoint(folder=folder, filename=self.best_model_filename,
                                                   iteration=self.iteration)
            if _dist():
                dist.barrier()
            self.best_model_manager.load_checkpoint(folder=folder, filename=self.best_model_filename)
        self.last_eval = res
        self.log(f"evaluation: candidate {res['wins']} best {res['losses']} draws {res['draws']}, "
                 f"win rate {res['win_rate']:.3f} -> {'promoted' if res['passed'] else 'kept best'}")
        return res

    def save_buffer(self):
        if self.rank != 0:
            return
        c = self.self_play_config
        Path(c.get("replay_buffer_folder", ".")).mkdir(parents=True, exist_ok=True)
        rec = self.replay_buffer.records()
        buffer_io.save_compact(rec, self._buffer_path(), maxlen=self.replay_buffer.capacity)
        if c.get("export_reference_pickle"):
            buffer_io.export_reference_pickle(
                rec, os.path.join(c["replay_buffer_folder"], c.get("replay_buffer_filename", "replay_buffer.pkl")),
                self.replay_buffer.capacity)

    def run_training_loop(self):
        c = self.self_play_config
        folder = c["checkpoint_folder"]
        resume = "latest_candidate.pth.tar"
        loaded, self.start_iteration = self.model_manager.load_checkpoint(folder=folder, filename=resume)
        if not loaded:
            self.start_iteration = 0
        history = []
        for it in range(self.start_iteration, c["num_iterations"]):
            self.iteration = it
            num = it + 1
            t0 = time.time()
            self.execute_self_play_phase(self.best_model_manager)
            self.execute_training_phase()
            self.model_manager.step_scheduler()
            if self.rank == 0:
                self.model_manager.save_checkpoint(folder=folder, filename=resume, iteration=num)
            self.save_buffer()
            ev = None
            if num % c["eval_frequency"] == 0:
                ev = self.evaluate_model()
            history.append({"iteration": num, "self_play": self.last_self_play, "training": self.last_training,
                            "evaluation": ev, "seconds": time.time() - t0})
        return history
