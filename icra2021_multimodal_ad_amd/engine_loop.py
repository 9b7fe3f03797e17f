"""Minimal ignite-free event loop used by the reference's driver
(novelty_detection.py:88-127 uses pytorch-ignite's Engine / Events /
RunningAverage, which is not installed here).  Semantics kept: process_fn
(engine, batch) per iteration, EPOCH_COMPLETED handlers, and RunningAverage
(alpha=0.98, reset at each epoch start, first value taken as-is)."""


class Events:
    STARTED = "started"
    EPOCH_STARTED = "epoch_started"
    ITERATION_COMPLETED = "iteration_completed"
    EPOCH_COMPLETED = "epoch_completed"
    COMPLETED = "completed"


class State:
    def __init__(self):
        self.epoch = 0
        self.iteration = 0
        self.output = None
        self.metrics = {}
        self.max_epochs = 0


class Engine:
    def __init__(self, process_fn):
        self._process_fn = process_fn
        self._handlers = {}
        self.state = State()

    def add_event_handler(self, event, handler, *args, **kwargs):
        self._handlers.setdefault(event, []).append((handler, args, kwargs))

    def on(self, event, *args, **kwargs):
        def deco(fn):
            self.add_event_handler(event, fn, *args, **kwargs)
            return fn
        return deco

    def _fire(self, event):
        for fn, args, kwargs in self._handlers.get(event, []):
            fn(self, *args, **kwargs)

    def run(self, data, max_epochs=1):
        self.state = State()
        self.state.max_epochs = max_epochs
        self._fire(Events.STARTED)
        for _ in range(max_epochs):
            self.state.epoch += 1
            self._fire(Events.EPOCH_STARTED)
            for batch in data:
                self.state.iteration += 1
                self.state.output = self._process_fn(self, batch)
                self._fire(Events.ITERATION_COMPLETED)
            self._fire(Events.EPOCH_COMPLETED)
        self._fire(Events.COMPLETED)
        return self.state


class RunningAverage:
    """ignite.metrics.RunningAverage(output_transform=...) on a scalar output."""

    def __init__(self, output_transform=lambda x: x, alpha=0.98):
        self.alpha = alpha
        self.output_transform = output_transform

    def attach(self, engine, name):
        state = {"v": None}

        def reset(eng):
            state["v"] = None

        def update(eng):
            val = float(self.output_transform(eng.state.output))
            state["v"] = val if state["v"] is None else state["v"] * self.alpha + (1 - self.alpha) * val
            eng.state.metrics[name] = state["v"]

        engine.add_event_handler(Events.EPOCH_STARTED, reset)
        engine.add_event_handler(Events.ITERATION_COMPLETED, update)
