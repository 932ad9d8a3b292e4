"""BatchedEnv: N Harmonies boards resident in HBM, stepped by HIP kernels.

This is the batched form of the reference env surface
(harmonies_engine.py: HarmoniesGameState() :66-79, get_legal_moves :145-208,
apply_move :210-298, calculate_score_for_player :357-367) and of the
encoder (process_game_state.py:15-137).  Every method enqueues work on the
current torch stream through libhz.so; nothing is computed on the host.
"""
import torch

from . import _native as nat
from .state import WORDS

ACTION_SIZE = 143


class BatchedEnv:
    def __init__(self, n_boards, seed_base=0, device="cuda"):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise nat.NativeError("BatchedEnv needs a GPU device (HIP); there is no CPU fallback")
        self.n = int(n_boards)
        L = nat.lib()
        with torch.cuda.device(self.device):
            self._h = L.hz_env_create(self.n, seed_base, nat.stream_ptr(self.device))
        if not self._h:
            raise nat.NativeError("hz_env_create failed")
        self.seed_base = seed_base
        self.epoch = 0  # bumped by every call that can start games (reset, rollout, import_state)
        self._mask = torch.zeros(self.n, 3, dtype=torch.int64, device=self.device)
        self._count = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self._status = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self._score = torch.zeros(self.n, 2, dtype=torch.int32, device=self.device)
        # hz_play's wait-error word (hz_env_set_error_word): a pipeline wave
        # that gave up waiting ORs a bit into it; rollout() looks at the last
        # call's copy once it has landed, check_errors() waits for it
        self.wait_err = torch.zeros(1, dtype=torch.int32, device=self.device)
        nat.check(L.hz_env_set_error_word(self._h, nat.ptr(self.wait_err)), "hz_env_set_error_word")
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_ev = None
        self._err_calls = 0

    # -- plumbing ----------------------------------------------------------
    def _sync_stream(self):
        nat.lib().hz_env_set_stream(self._h, nat.stream_ptr(self.device))

    def _out(self, t, shape, dtype, name):
        """A caller-supplied buffer the kernels write: checked before its
        pointer goes to the library (which trusts the size), None passes."""
        if t is None:
            return None
        dev = t.device if isinstance(t, torch.Tensor) else None
        if (dev is None or dev.type != "cuda" or (self.device.index is not None and dev.index != self.device.index)
                or t.dtype != dtype or tuple(t.shape) != tuple(shape) or not t.is_contiguous()):
            got = f"{t.dtype} {tuple(t.shape)} on {dev}" if dev is not None else type(t).__name__
            raise ValueError(f"{name}: expected a contiguous {dtype} tensor of shape {tuple(shape)} on "
                             f"{self.device}, got {got}")
        return t

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            nat.lib().hz_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_seed_ahead(self, enable, draws=24):
        """hz_play's concurrent next-episode preparation (seeding + the first
        `draws` pile draws) on/off; results are identical either way."""
        nat.check(nat.lib().hz_env_set_seed_ahead(self._h, int(draws) if enable else 0), "hz_env_set_seed_ahead")

    def set_auto_ahead(self, enable):
        """hz_rollout(auto_reset)'s episodes prepared ahead on/off
        (hz_env_set_auto_ahead); results are identical either way."""
        nat.check(nat.lib().hz_env_set_auto_ahead(self._h, int(bool(enable))), "hz_env_set_auto_ahead")

    def set_pipeline(self, pipeline):
        """hz_play's pipeline: 2 (the default) = every game spread over thirteen
        consecutive calls (k_play2), 1 = chance-ahead (k_rollout); results
        are identical either way (hz_env_set_pipeline)."""
        L = nat.lib()
        if not hasattr(L, "hz_env_set_pipeline") and int(pipeline) == 1:
            return  # (an older A/B build: pipeline 1 is all it has)
        nat.check(L.hz_env_set_pipeline(self._h, int(pipeline)), "hz_env_set_pipeline")

    # -- env surface ---------------------------------------------------------
    def reset(self, sel=None, seeds=None):
        """HarmoniesGameState() on every board (or on boards where sel != 0)."""
        self._sync_stream()
        self.epoch += 1
        if sel is not None:
            sel = sel.to(device=self.device, dtype=torch.uint8).contiguous()
        if seeds is not None:
            seeds = seeds.to(device=self.device, dtype=torch.int64).contiguous()
        nat.check(nat.lib().hz_reset(self._h, nat.ptr(sel), nat.ptr(seeds)), "hz_reset")

    def replenish(self, sel=None):
        """_replenish_piles on every (selected) board."""
        self._sync_stream()
        sel = None if sel is None else sel.to(device=self.device, dtype=torch.uint8).contiguous()
        nat.check(nat.lib().hz_replenish(self._h, nat.ptr(sel)), "hz_replenish")

    def end_turn(self, sel=None):
        """_end_turn_actions on every (selected) board."""
        self._sync_stream()
        sel = None if sel is None else sel.to(device=self.device, dtype=torch.uint8).contiguous()
        nat.check(nat.lib().hz_end_turn(self._h, nat.ptr(sel)), "hz_end_turn")

    def legal_mask(self, out=None, count=None):
        """143-bit legal-action mask per board, int64 [n, 3] (bit i of word w
        = action 64*w + i) and the number of legal actions int32 [n]."""
        self._sync_stream()
        out = self._mask if out is None else self._out(out, (self.n, 3), torch.int64, "out")
        count = self._count if count is None else self._out(count, (self.n,), torch.int32, "count")
        nat.check(nat.lib().hz_legal_mask(self._h, nat.ptr(out), nat.ptr(count)), "hz_legal_mask")
        return out, count

    def legal_actions(self, out=None, count=None):
        """Boolean [n, 143] legal-action mask (get_legal_moves through
        get_action_index, one launch: hz_legal_actions) and the legal counts
        int32 [n]."""
        self._sync_stream()
        out = (torch.empty(self.n, ACTION_SIZE, dtype=torch.bool, device=self.device) if out is None
               else self._out(out, (self.n, ACTION_SIZE), torch.bool, "out"))
        count = self._count if count is None else self._out(count, (self.n,), torch.int32, "count")
        nat.check(nat.lib().hz_legal_actions(self._h, nat.ptr(out), nat.ptr(count)), "hz_legal_actions")
        return out

    def step(self, actions, status=None):
        """apply_move per board (actions int16 [n], <0 = no-op); int32 status."""
        self._sync_stream()
        actions = actions.to(device=self.device, dtype=torch.int16).contiguous()
        status = self._status if status is None else self._out(status, (self.n,), torch.int32, "status")
        nat.check(nat.lib().hz_step(self._h, nat.ptr(actions), nat.ptr(status)), "hz_step")
        return status

    def score(self, parts=False):
        """calculate_score_for_player for both players: int32 [n, 2]
        (and [n, 2, 5] per-habitat parts when parts=True)."""
        self._sync_stream()
        out = self._score
        pt = torch.zeros(self.n, 2, 5, dtype=torch.int32, device=self.device) if parts else None
        nat.check(nat.lib().hz_score(self._h, nat.ptr(out), nat.ptr(pt)), "hz_score")
        return (out, pt) if parts else out

    def encode(self, idx=None, board=None, glob=None):
        """create_state_tensors for boards idx (default all): f32 [m,38,5,7], [m,42]."""
        self._sync_stream()
        if idx is not None:
            idx = idx.to(device=self.device, dtype=torch.int32).contiguous()
            m = idx.numel()
        else:
            m = self.n
        if board is None:
            board = torch.empty(m, 38, 5, 7, dtype=torch.float32, device=self.device)
        if glob is None:
            glob = torch.empty(m, 42, dtype=torch.float32, device=self.device)
        nat.check(nat.lib().hz_encode(self._h, nat.ptr(idx), m, nat.ptr(board), nat.ptr(glob)), "hz_encode")
        return board, glob

    def rule_actions(self, mask=None, count=None, out=None):
        """The build-defined deterministic policy (splitmix64 rule)."""
        self._sync_stream()
        if mask is None:
            mask, count = self.legal_mask()
        mask = self._out(mask, (self.n, 3), torch.int64, "mask")
        count = self._out(count, (self.n,), torch.int32, "count")
        out = (torch.empty(self.n, dtype=torch.int16, device=self.device) if out is None
               else self._out(out, (self.n,), torch.int16, "out"))
        nat.check(nat.lib().hz_rule_actions(self._h, nat.ptr(mask), nat.ptr(count), nat.ptr(out)),
                  "hz_rule_actions")
        return out

    def rule_ply(self, mask=None, count=None, action=None, status=None):
        """legal_mask -> rule_actions -> step for every board in one launch
        (hz_rule_ply); the given output tensors get what the three calls
        would write."""
        self._sync_stream()
        mask = self._out(mask, (self.n, 3), torch.int64, "mask")
        count = self._out(count, (self.n,), torch.int32, "count")
        action = self._out(action, (self.n,), torch.int16, "action")
        status = self._out(status, (self.n,), torch.int32, "status")
        nat.check(nat.lib().hz_rule_ply(self._h, nat.ptr(mask), nat.ptr(count), nat.ptr(action), nat.ptr(status)),
                  "hz_rule_ply")

    def greedy_actions(self, sel=None, out=None):
        """choose_move_greedy (evaluation.py:137-196) for every board (or where
        sel != 0): int16 [n], -1 where finished / unselected.  Consumes the
        chance streams like the reference's simulated apply_move calls; apply
        the result with step()."""
        self._sync_stream()
        if sel is not None:
            sel = sel.to(device=self.device, dtype=torch.uint8).contiguous()
        out = (torch.empty(self.n, dtype=torch.int16, device=self.device) if out is None
               else self._out(out, (self.n,), torch.int16, "out"))
        nat.check(nat.lib().hz_greedy_actions(self._h, nat.ptr(sel), nat.ptr(out)), "hz_greedy_actions")
        return out

    def rollout(self, max_plies, auto_reset=False, record=False, games_done=None, steps_done=None, reset=False):
        """Fused rule-driven play of up to max_plies plies per board
        (reset=True: start every board's next game first, in the same launch)."""
        self._sync_stream()
        self.epoch += 1
        traj = None
        if record:
            traj = (torch.zeros(max_plies, WORDS, self.n, dtype=torch.int64, device=self.device),
                    torch.zeros(max_plies, self.n, 3, dtype=torch.int64, device=self.device),
                    torch.full((max_plies, self.n), -1, dtype=torch.int16, device=self.device))
        games_done = (torch.zeros(self.n, dtype=torch.int32, device=self.device) if games_done is None
                      else self._out(games_done, (self.n,), torch.int32, "games_done"))
        steps_done = (torch.zeros(self.n, dtype=torch.int32, device=self.device) if steps_done is None
                      else self._out(steps_done, (self.n,), torch.int32, "steps_done"))
        ts, tm, ta = traj if traj else (None, None, None)
        fn = nat.lib().hz_play if reset else nat.lib().hz_rollout
        nat.check(fn(self._h, int(max_plies), int(bool(auto_reset)), nat.ptr(ts), nat.ptr(tm), nat.ptr(ta),
                     nat.ptr(games_done), nat.ptr(steps_done)), "hz_play" if reset else "hz_rollout")
        self._poll_errors()
        return games_done, steps_done, traj

    POLL_EVERY = 32  # rollout calls between two queued error-word copies

    def _poll_errors(self):
        """After a rollout launch: if the last queued error-word copy has
        landed, raise on it; every POLL_EVERY calls queue a new copy (no host
        wait).  check_errors() waits and checks everything queued so far."""
        ev = self._err_ev
        if ev is not None and ev.query():
            self._err_ev = None
            self._raise_wait_error(int(self._err_host[0]))
        self._err_calls += 1
        # (a copy and an event on the stream every POLL_EVERY calls, not
        # every call: back-to-back launches stay back to back)
        if self._err_ev is None and self._err_calls >= self.POLL_EVERY:
            self._err_calls = 0
            self._err_host.copy_(self.wait_err, non_blocking=True)
            self._err_ev = torch.cuda.Event()
            self._err_ev.record()

    def _raise_wait_error(self, bits):
        if bits:
            self.wait_err.zero_()
            raise nat.NativeError(
                f"hz_play: a pipeline wave gave up waiting for its publisher (error bits {bits:#x}: 1 = seed-stage "
                "rows, 2 = k_play2 twist); the streams of that call are not trustworthy")

    def check_errors(self):
        """Wait for the work queued so far and raise NativeError if any
        hz_play / hz_rollout wait gave up since the last check."""
        self._err_ev = None
        bits = int(self.wait_err.item())
        self._raise_wait_error(bits)

    def set_spin_limit(self, limit):
        """Test knob (hz_env_set_spin_limit): 0 = default bound."""
        nat.check(nat.lib().hz_env_set_spin_limit(self._h, int(limit)), "hz_env_set_spin_limit")

    # -- state transfer -------------------------------------------------------
    def export_state(self, with_mt=False):
        """int64 [6, n] state words (+ uint32-as-int32 [n, 624] MT words and
        int32 [n] CPython indices when with_mt: random.setstate((3, tuple(mt[b]) +
        (idx[b],), None)) continues board b's stream)."""
        self._sync_stream()
        st = torch.empty(WORDS, self.n, dtype=torch.int64, device=self.device)
        mt = idx = None
        if with_mt:
            mt = torch.empty(self.n, 624, dtype=torch.int32, device=self.device)
            idx = torch.empty(self.n, dtype=torch.int32, device=self.device)
        nat.check(nat.lib().hz_export_state(self._h, nat.ptr(st), nat.ptr(mt), nat.ptr(idx)), "hz_export_state")
        return (st, mt, idx) if with_mt else st

    def import_state(self, state, mt=None, mt_index=None):
        self._sync_stream()
        self.epoch += 1
        state = state.to(device=self.device, dtype=torch.int64).contiguous()
        if mt is not None:
            mt = mt.to(device=self.device, dtype=torch.int32).contiguous()
            mt_index = mt_index.to(device=self.device, dtype=torch.int32).contiguous()
        nat.check(nat.lib().hz_import_state(self._h, nat.ptr(state), nat.ptr(mt), nat.ptr(mt_index)),
                  "hz_import_state")

    def done(self):
        """is_game_over() per board (bool [n]) from the state words."""
        misc = self.export_state()[5]
        over = (misc >> 45) & 1
        win = (misc >> 46) & 3
        return (over == 1) & (win != 0)


_BIT = None


def unpack_mask(mask):
    """int64 [n, 3] packed mask -> bool [n, 143]."""
    global _BIT
    if _BIT is None or _BIT.device != mask.device:
        _BIT = torch.arange(64, device=mask.device, dtype=torch.int64)
    bits = (mask.unsqueeze(-1) >> _BIT) & 1  # [n, 3, 64]
    return bits.reshape(mask.shape[0], 192)[:, :ACTION_SIZE].bool()
