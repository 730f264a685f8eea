"""aiforearth_api_platform_amd — MI355X-native async inference-serving platform.

A from-scratch re-design of the AI for Earth API Platform (reference:
CSA-DanielVillamizar/AIforEarth-API-Platform) for one node of 8x AMD Instinct MI355X:

* ``api``      drop-in-model decorator API (``APIService``) and ``TaskManager`` (reference L3)
* ``gateway``  HTTP front end + in-process task control plane (reference L7/L6/L5)
* ``store``    native C++ task store + dispatch queue (Redis / Service Bus replacement)
* ``sched``    dispatchers (queue pull / webhook push) and the dynamic GPU batcher (reference L4)
* ``runtime``  per-GPU engines and worker pool, pipeline stages, spatial parallelism (reference L1)
* ``models``   ResNet-50, Faster-RCNN R50-FPN, U-Net, crop classifier on NHWC bf16
* ``ops``      hand-written CDNA4 HIP kernels (``csrc/kernels``) behind a torch-tensor API
* ``parallel`` torch.distributed (RCCL over xGMI) helpers: p2p hand-off, halo exchange, broadcast
* ``utils``    structured logging, metrics registry, tracing
"""
__version__ = "0.1.0"
