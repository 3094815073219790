"""In-stream kernel timing for the bench roofline: a pair of HIP events recorded around one chosen kernel of
every training step (mplc_cnn_train_t.prof_kernel), on the stream the kernel is launched on."""


class KernelTimer:
    def __init__(self, kernel):
        self.kernel = kernel
        self.events = []
        self.samples = []

    def pair(self):
        import torch
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        # materialise the underlying hipEvent_t (torch creates it lazily on first record); the library
        # re-records both inside the step, in stream order, so elapsed_time covers exactly the kernel
        a.record()
        b.record()
        self.events.append((a, b))
        return a.cuda_event, b.cuda_event

    def total_ms(self):
        import torch
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) for a, b in self.events)

    def launches(self):
        return len(self.events)
