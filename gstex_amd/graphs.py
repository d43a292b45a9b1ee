"""hipGraph capture of whole single-GPU training steps (not in the reference, whose step is eager PyTorch).

A read-back-free GStexTrainer step (pair_capacity, defer_texture, fused Adam: no host synchronisation inside the step,
gstex_amd.model) is a fixed sequence of ~40 launches.  Enqueued eagerly it costs ~1.1 ms of host time per step (Python,
autograd and ~40 hipLaunchKernel calls), which the device hides in steady state (the host runs ahead of a 2.3 ms
step) but not after a synchronisation: the first step then waits ~0.5 ms for the host to reach its raster forward.
StepGraphs captures one step per slot (e.g. per camera pose of the loop's cycle) into a hipGraph and replays it with
one hipGraphLaunch, so the device starts every step, the first one included, with the whole step queued.

What a replay changes versus its capture, and how:
  * the Adam bias corrections of step t: read on the device from per-parameter tables (optim.AdamSchedule,
    gstex_adam_step_scheduled) at a row the graph's own counter advances each replay -- the same fp32 scalars the
    eager step passes;
  * the host state an eager step advances (trainer.step, each parameter's Adam step count, the deferred texel update
    left pending): advanced by replay() as the eager step would;
  * kernel timing (ops.set_kernel_timing): the timed launches are captured between event-record nodes
    (gstex_event_record_external) that replay() points at a fresh event pair each time;
  * the pair-capacity guard: a capture sizes the pair buffers from the current capacity and reports the pair total
    into the slot's own host word; poll() reads it between replays and marks the graphs stale (re-captured at the next
    replay) when the capacity has to grow.  An overflowing replay skips its update on the device, as an eager step.
Everything else (camera, parameters, buffers) is the same memory every replay: a rechart or any other change of the
parameter tensors needs capture() again.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib, ops
from .optim import AdamSchedule, FusedAdam


_UPLOAD = os.environ.get("GSTEX_GRAPH_UPLOAD", "current")  # hipGraphUpload after instantiation: none | capture | current


class _Slot:
    __slots__ = ("graph", "exec_ptr", "timing", "current", "pending", "capacity", "updated")


class StepGraphs:
    """Captured training steps of `trainer`, one per slot: step_fn(k) enqueues slot k's step on the current stream
    (e.g. zero_grad, forward_backward on pose k, optimizer_step).  capture() once the pair capacity is sized (one eager
    step) and after every change of the parameter tensors; then replay(k) in place of step_fn(k).  `timed`: C-ABI
    entry points (ops.set_kernel_timing names) to time inside the graphs."""

    def __init__(self, trainer, step_fn, n_slots: int, timed=(), rows: int = 8192):
        self.tr = trainer
        # one pair-capacity flag slot for every step (gstex_amd.model: step k's flag is read by its head update and, at
        # the top of step k + 1, by its deferred texel update, before step k + 1's scan overwrites it): a captured
        # step then reads the flag of whichever step (eager or replayed) ran before it
        trainer.single_flag = True
        self.step_fn = step_fn
        self.n = int(n_slots)
        self.timed = set(timed)
        self.rows = int(rows)
        self.slots: list = [None] * self.n
        self.schedule = None
        self._pool = None
        self._stream = None
        self.replays = 0
        self._row0 = 0  # replays taken off the schedule's counter by AdamSchedule.shift
        self._polls = []  # (event, [(slot, trainer step), ...]) of replays whose pair totals have not been read
        self._unpolled = []  # replays since the last poll event
        self._expected_step = None  # trainer.step after the last capture / replay (eager steps since: stale)
        self.stale = False
        self._host_words = self._dev_words = None

    # ------------------------------------------------------------------ host state of a step
    def _params(self):
        return [p for g in self.tr.optimizer.param_groups for p in g["params"]]

    def _snapshot(self):
        tr, opt = self.tr, self.tr.optimizer
        return dict(step=tr.step, pending=tr._pending_tex, sink=tr._sink_fresh, skipped=list(tr.skipped_steps),
                    grads={id(p): p.grad for p in self._params()},
                    steps={id(p): opt.state[p]["step"] for p in self._params() if "step" in opt.state.get(p, {})})

    def _restore(self, s):
        tr, opt = self.tr, self.tr.optimizer
        tr.step, tr._pending_tex, tr._sink_fresh = s["step"], s["pending"], s["sink"]
        tr._pending_collective = False
        tr.skipped_steps[:] = s["skipped"]
        for p in self._params():
            p.grad = s["grads"][id(p)]
            if id(p) in s["steps"]:
                opt.state[p]["step"] = s["steps"][id(p)]

    # ------------------------------------------------------------------ capture
    def _check(self):
        tr = self.tr
        if not (isinstance(tr.optimizer, FusedAdam) and tr.defer_texture and tr.pairs is not None):
            raise RuntimeError("StepGraphs: needs a read-back-free trainer (fused Adam, defer_texture, pair_capacity)")
        if tr.texture_grad_route is not None or tr._pending_collective:
            raise RuntimeError("StepGraphs: single-GPU steps only (a GradSync step has collectives)")
        if tr.pairs.capacity <= 0:
            raise RuntimeError("StepGraphs: run one eager step first (it sizes the pair capacity)")

    def _reset(self):
        """Drop every slot and start a new schedule (after a device synchronisation: replays of the old graphs may be
        in flight, and their memory pool goes with them)."""
        dev = self.tr.device
        torch.cuda.synchronize(dev)
        self._poll_all()
        self.slots = [None] * self.n
        self._pool = None
        if self._host_words is None:
            h, d = ctypes.c_void_p(), ctypes.c_void_p()
            _lib.call("gstex_host_words_alloc", self.n, ctypes.byref(h), ctypes.byref(d))
            self._host_words, self._dev_words = h.value, d.value
            self._words = (ctypes.c_int32 * self.n).from_address(self._host_words)
        self.schedule = AdamSchedule(self.tr.optimizer, dev, self.rows)
        self.replays, self._row0 = 0, 0
        self.stale = False
        self._expected_step = self.tr.step

    def capture(self, slots=None):
        """Capture the steps of `slots` (default: every slot) back to back, after dropping every graph captured before
        (a device synchronisation, a fresh memory pool and a fresh schedule).  Captures are never interleaved with
        replays of graphs that share their pool: that pattern (a slot captured lazily after other slots of the same
        pool had been replayed) faulted the GPU on a later replay in round 5, while back-to-back captures replay
        correctly.  The device idles for the few ms of a capture (its clock then takes several steps to ramp back
        up): capture outside the timed region."""
        self._check()
        want = sorted(set(range(self.n) if slots is None else slots) |
                      {k for k, sl in enumerate(self.slots) if sl is not None})
        self._reset()
        for k in want:
            self._capture_slot(k)

    def _capture_slot(self, k: int):
        tr = self.tr
        dev = tr.device
        snap = self._snapshot()
        n_params = len(self._params())
        if self._stream is None:
            self._stream = torch.cuda.Stream(dev)
        stream = self._stream
        stream.wait_stream(torch.cuda.current_stream(dev))
        tr.optimizer.schedule = self.schedule
        try:
            tr.pairs.graph_word = self._dev_words + 4 * k
            ops._CAPTURE_TIMED, ops._CAPTURE_TIMING = set(self.timed), []
            self.schedule.reset_updates()
            g = torch.cuda.CUDAGraph(keep_graph=True)
            # (torch.cuda.graph: the device synchronised and the caches emptied first; one pool for all slots, which
            # are replayed one at a time on one stream)
            with torch.cuda.graph(g, pool=self._pool, stream=stream):
                self.step_fn(k)
                self.schedule.counter.add_(1)  # the next replay reads the next table row
            timing = ops._CAPTURE_TIMING
            ops._CAPTURE_TIMED = ops._CAPTURE_TIMING = None
            if not self.schedule.updates or set(self.schedule.updates.values()) != {1}:
                raise RuntimeError("StepGraphs: the captured step must update each parameter at most once "
                                   f"(got {sorted(self.schedule.updates.values())} over {n_params} parameters)")
            updated = set(self.schedule.updates)  # (parameters without a gradient, e.g. features_dc, are not)
            if self._pool is None:
                self._pool = g.pool()
            g.instantiate()
            if _UPLOAD == "capture":
                _lib.call("gstex_graph_upload", g.raw_cuda_graph_exec(), stream.cuda_stream)
            elif _UPLOAD == "current":  # the stream the replays will run on
                _lib.call("gstex_graph_upload", g.raw_cuda_graph_exec(), torch.cuda.current_stream(dev).cuda_stream)
            s = _Slot()
            s.graph, s.exec_ptr = g, g.raw_cuda_graph_exec()
            s.timing = []
            for key, a, b in timing:
                evs = (ctypes.c_void_p * 2)(a.handle, b.handle)
                nodes = (ctypes.c_void_p * 2)()
                _lib.call("gstex_graph_event_nodes", g.raw_cuda_graph(), evs, 2, nodes)
                s.timing.append((key, a, b, nodes[0], nodes[1]))
            s.current = None  # the timing events the nodes record into now (None: the capture's own pair)
            s.pending = tr._pending_tex  # the step's deferred texel update, run eagerly if no replay follows
            s.capacity = tr.pairs.capacity
            s.updated = updated
            self.slots[k] = s
        finally:
            tr.optimizer.schedule = None
            tr.pairs.graph_word = None
            ops._CAPTURE_TIMED = ops._CAPTURE_TIMING = None
            self._restore(snap)
        torch.cuda.current_stream(dev).wait_stream(stream)

    # ------------------------------------------------------------------ replay
    def _point_timing(self, s: _Slot):
        timing_on = ops._TIMING is not None
        if timing_on and s.timing:
            cur = []
            for key, a, b, na, nb in s.timing:
                ea, eb = _lib.TimingEvent(), _lib.TimingEvent()
                _lib.call("gstex_graph_exec_set_event", s.exec_ptr, na, ea.handle)
                _lib.call("gstex_graph_exec_set_event", s.exec_ptr, nb, eb.handle)
                if key in ops._TIMED:
                    ops._TIMING.setdefault(key, []).append((ea, eb))
                cur.append((ea, eb))
            s.current = cur
        elif s.current is not None:  # back to the capture's pair: a finished timing session's events stay intact
            for key, a, b, na, nb in s.timing:
                _lib.call("gstex_graph_exec_set_event", s.exec_ptr, na, a.handle)
                _lib.call("gstex_graph_exec_set_event", s.exec_ptr, nb, b.handle)
            s.current = None

    def replay(self, k: int):
        """Slot k's step, one hipGraphLaunch on the current stream; host state advanced as the eager step's."""
        if self._expected_step is not None and self.tr.step != self._expected_step:
            self.stale = True  # eager steps since the last capture / replay: re-captured (the rows follow the steps)
        if self.stale or self.schedule is None or self.slots[k] is None:
            self.capture([k])
        tr, opt = self.tr, self.tr.optimizer
        s = self.slots[k]
        while self.replays - self._row0 >= self.rows - 1:  # slide the bias-correction tables before the rows run out
            n = self.rows // 2
            self.schedule.shift(n)
            self._row0 += n
        self._point_timing(s)
        s.graph.replay()
        self.replays += 1
        tr._pending_tex, tr._pending_collective, tr._sink_fresh = s.pending, False, True
        for p in self._params():
            if id(p) in s.updated:
                opt.state[p]["step"] += 1
        self._unpolled.append((k, tr.step))
        tr.step += 1
        self._expected_step = tr.step
        if len(self._unpolled) >= self.n:  # one poll event per cycle of slots (an event is a marker packet, ~4 us)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(tr.device))
            self._polls.append((ev, self._unpolled))
            self._unpolled = []
        self.poll()

    # ------------------------------------------------------------------ pair totals
    def _absorb(self, k: int, step: int):
        pairs = self.tr.pairs
        total = int(self._words[k])
        pairs.last_total = total
        pairs.max_total = max(pairs.max_total, total)
        if total > self.slots[k].capacity:  # the replay's update was skipped on the device (guarded Adam)
            pairs.overflows.append(step)
            self.tr.skipped_steps.append(step)
        if total > pairs.grow_at * pairs.capacity:
            pairs.capacity = max(pairs.capacity, int(pairs.headroom * total) + pairs.slack)
        if pairs.capacity > self.slots[k].capacity:
            self.stale = True  # re-captured (larger pair buffers) at the next replay

    def poll(self):
        """Read the pair totals of the replays the stream has passed (non-blocking).  A slot's word holds its latest
        replay's total: read late, the totals of earlier replays of that slot are not seen (the device-side guard
        still skips their updates)."""
        while self._polls and self._polls[0][0].query():
            for k, step in self._polls.pop(0)[1]:
                self._absorb(k, step)

    def _poll_all(self):
        """(after a device synchronisation)"""
        for _, done in self._polls:
            for k, step in done:
                self._absorb(k, step)
        for k, step in self._unpolled:
            self._absorb(k, step)
        self._polls, self._unpolled = [], []

    @property
    def captured(self) -> int:
        return sum(s is not None for s in self.slots)

    def close(self):
        """Wait for the replays, read their pair totals and drop the graphs (their memory pool is released)."""
        if self.captured:
            torch.cuda.synchronize(self.tr.device)
            self._poll_all()
        self.slots = [None] * self.n
        self.schedule = self._pool = None
        if self._host_words is not None:
            _lib.load().gstex_host_words_free(self._host_words)
            self._host_words = self._dev_words = None
