"""In-stream kernel timing for the bench roofline: HIP events recorded by the library around the kernels of
every training step (mplc_cnn_train_t.prof_kernel), on the stream the kernels are launched on.

KernelTimer("conv_bwd_data") times one kernel; KernelTimer("all", names) times every launch of the step
(prof_kernel = MPLC_PROF_ALL, the event handles passed as arrays indexed by kernel id).  Completed event pairs
are folded into running totals with non-blocking queries, so a long timed region keeps only the last few
steps' events alive and never synchronises.

With stash=True the model also keeps a device copy of each step's schedule (cnt, adam_t), from which the
algorithmic units of every kernel (samples; the dense kernels' HBM bytes, which depend on the Adam step) are
counted exactly after the timed region (MnistModel.algorithmic_units)."""
import ctypes

PROF_ALL = -1  # include/mplc_hip_cnn.h MPLC_PROF_ALL


class KernelTimer:
    def __init__(self, kernel, names=None, stash=False, per_launch=()):
        self.kernel = kernel
        self.want_stash = stash
        self.per = {n: [] for n in per_launch}  # every launch's ms, in launch order, for these kernel names
        self.names = list(names) if names is not None else [kernel]
        self.pending = []            # [(name, begin, end)]
        self.ms = {n: 0.0 for n in self.names}
        self.count = {n: 0 for n in self.names}
        self._keep = []              # ctypes arrays passed to the library for the pending steps
        self.stash = []              # per step: device copies of the schedule tensors the model accounts from

    @property
    def all(self):
        return self.kernel == "all"

    def _event_pair(self):
        import torch
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        # materialise the underlying hipEvent_t (torch creates it lazily on first record); the library
        # re-records both inside the step, in stream order, so elapsed_time covers exactly the kernel
        a.record()
        b.record()
        return a, b

    def _fold(self, block=False):
        keep = []
        for name, a, b in self.pending:
            if block or b.query():
                if name in self.ms:
                    ms = a.elapsed_time(b)
                    self.ms[name] += ms
                    self.count[name] += 1
                    if name in self.per:
                        self.per[name].append(ms)
            else:
                keep.append((name, a, b))
        self.pending = keep
        if len(self._keep) > 64:
            self._keep = self._keep[-64:]

    def pair(self):
        """(begin, end) handles for one step: hipEvent_t values, or for "all" pointers to hipEvent_t arrays
        indexed by kernel id (ids = the model's KERNEL_IDS)."""
        if len(self.pending) > 256:
            self._fold()
        if not self.all:
            a, b = self._event_pair()
            self.pending.append((self.kernel, a, b))
            return a.cuda_event, b.cuda_event
        # the library records ev[k] for EVERY kernel id of the step (mplc_cnn_train_step / mplc_cifar_train_step),
        # so the arrays cover all of the model's ids with live events; ids outside `names` are recorded, not counted
        n = max(self.all_ids.values()) + 1
        begin = (ctypes.c_void_p * n)()
        end = (ctypes.c_void_p * n)()
        for name, k in self.all_ids.items():
            a, b = self._event_pair()
            begin[k], end[k] = a.cuda_event, b.cuda_event
            self.pending.append((name, a, b))
        assert all(begin[k] and end[k] for k in range(1, n)), "every kernel id of the step needs an event pair"
        self._keep.append((begin, end))
        return ctypes.addressof(begin), ctypes.addressof(end)

    def bind(self, kernel_ids):
        """Kernel ids of the model being timed (its KERNEL_IDS: ids 1..K, every launch of the step)."""
        if sorted(kernel_ids.values()) != list(range(1, len(kernel_ids) + 1)):
            raise ValueError("KERNEL_IDS must number the step's launches 1..K")
        self.all_ids = dict(kernel_ids)
        self.ids = {n: kernel_ids[n] for n in self.names}
        return self

    def stash_step(self, *tensors):
        """Keep device copies of a step's schedule tensors (cnt, adam_t) for the algorithmic-unit count made
        after the timed region (a copy per tensor and step: no host sync inside the region)."""
        self.stash.append(tuple(t.clone() for t in tensors))

    def total_ms(self, name=None):
        import torch
        torch.cuda.synchronize()
        self._fold(block=True)
        return self.ms[name or self.kernel]

    def launches(self, name=None):
        self._fold(block=True)
        return self.count[name or self.kernel]


class StashOnly:
    """A profiler that times nothing and only stashes every step's schedule (bench.py under rocprofv3 --pmc, where
    no HIP event may be recorded): the algorithmic units of ALL launches of the run, to set beside the counters'
    bytes of the same launches."""
    all = False
    want_stash = True

    def __init__(self, kernel):
        self.kernel = kernel  # any kernel of the model: the library records nothing (NULL events)
        self.stash = []
        self.evals = []  # (models, samples, sample chunks) of every evaluation launch group (CifarModel.evaluate)

    def pair(self):
        return None, None

    def stash_step(self, *tensors):
        self.stash.append(tuple(t.clone() for t in tensors))

    def stash_eval(self, n_models, n_samples, chunks):
        self.evals.append((int(n_models), int(n_samples), int(chunks)))
