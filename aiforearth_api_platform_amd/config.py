"""Single configuration object for the platform.

Collapses the reference's three string-env tiers into one dataclass
(survey §5.6):

1. platform flags of ``InfrastructureDeployment/setup_env.sh:3-82`` (transport type, retry delay,
   max deliveries, Redis timeouts -> store/queue knobs),
2. function-app settings (``deploy_cache_manager.sh:36-150``, ``deploy_backend_queue_function.sh``),
3. container env of the Helm charts (``APIs/Charts/templates/async-gpu/templates/deployment.yaml:23-49``)
   read by ``APIs/1.0/base-py/ai4e_service.py:19-22,51``.

Precedence: explicit overrides (CLI flags) > environment variables > YAML file > defaults.
The container env names are kept verbatim; GPU knobs use the ``AI4E_`` prefix.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional


def _as_bool(v: Any) -> bool:
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() in ("1", "true", "yes", "on", "y")


@dataclass
class Config:
    # --- container runtime (ai4e_service.py / deployment.yaml) ---
    api_prefix: str = field(default="", metadata={"env": "API_PREFIX"})
    cache_connector_upsert_uri: str = field(default="", metadata={"env": "CACHE_CONNECTOR_UPSERT_URI"})
    cache_connector_get_uri: str = field(default="", metadata={"env": "CACHE_CONNECTOR_GET_URI"})
    current_processing_upsert_uri: str = field(default="", metadata={"env": "CURRENT_PROCESSING_UPSERT_URI"})
    # Reference default 'True' (ai4e_service.py:19). Parsed as a real bool here (Appendix B #2 fix).
    disable_current_request_metric: bool = field(default=True, metadata={"env": "DISABLE_CURRENT_REQUEST_METRIC"})
    service_cluster: str = field(default="undefined", metadata={"env": "SERVICE_CLUSTER"})
    service_owner: str = field(default="AI4E", metadata={"env": "SERVICE_OWNER"})
    service_name: str = field(default="ai4e-mi355x", metadata={"env": "SERVICE_NAME"})
    service_version: str = field(default="1.0", metadata={"env": "SERVICE_VERSION"})
    service_model_name: str = field(default="", metadata={"env": "SERVICE_MODEL_NAME"})
    service_model_framework: str = field(default="pytorch-rocm", metadata={"env": "SERVICE_MODEL_FRAMEWORK"})
    service_model_framework_version: str = field(default="", metadata={"env": "SERVICE_MODEL_FRAMEOWRK_VERSION"})
    service_model_version: str = field(default="", metadata={"env": "SERVICE_MODEL_VERSION"})
    service_container_name: str = field(default="", metadata={"env": "SERVICE_CONTAINER_NAME"})
    service_container_version: str = field(default="", metadata={"env": "SERVICE_CONTAINER_VERSION"})
    next_api_name_in_pipeline: str = field(default="", metadata={"env": "NEXT_API_NAME_IN_PIPELINE"})
    debug: bool = field(default=False, metadata={"env": "DEBUG"})
    # adaptive telemetry sampling of the structured logs (App Insights samplingSettings.maxTelemetryItemsPerSecond = 50,
    # ProcessManager/CacheManager/host.json:3-9): the emitted rate is held near this many items/s; 0 = keep everything
    telemetry_max_per_s: float = field(default=50.0, metadata={"env": "AI4E_TELEMETRY_MAX_PER_S"})
    # --- transport / dispatcher (setup_env.sh:65-74, BackendQueueProcessor/host.json) ---
    transport: str = field(default="inproc", metadata={"env": "AI4E_TRANSPORT"})  # inproc|queue|eventgrid
    queue_retry_delay_ms: int = field(default=60000, metadata={"env": "QUEUE_RETRY_DELAY_MS"})
    max_delivery_count: int = field(default=1440, metadata={"env": "SERVICEBUS_QUEUE_MAX_DELIVERY_COUNT"})
    queue_lock_duration_s: float = field(default=300.0, metadata={"env": "AI4E_QUEUE_LOCK_DURATION_S"})
    queue_max_size: int = field(default=0, metadata={"env": "AI4E_QUEUE_MAX_SIZE"})
    dispatch_concurrency: int = field(default=1, metadata={"env": "AI4E_DISPATCH_CONCURRENCY"})
    eventgrid_max_delivery_attempts: int = field(default=3, metadata={"env": "AI4E_EVENTGRID_MAX_ATTEMPTS"})
    eventgrid_event_ttl_s: float = field(default=300.0, metadata={"env": "AI4E_EVENTGRID_TTL_S"})
    # --- task store (Redis replacement) ---
    store_backend: str = field(default="native", metadata={"env": "AI4E_STORE_BACKEND"})  # native|python
    journal_path: str = field(default="", metadata={"env": "AI4E_JOURNAL"})
    finished_task_ttl_s: float = field(default=3600.0, metadata={"env": "AI4E_FINISHED_TASK_TTL_S"})
    evict_period_s: float = field(default=10.0, metadata={"env": "AI4E_EVICT_PERIOD_S"})
    # finished tasks (and their results) kept per endpoint and state regardless of age
    max_finished_tasks: int = field(default=4_000_000, metadata={"env": "AI4E_MAX_FINISHED_TASKS"})
    # request bodies up to this size are journaled as the task's _ORIG body (replayed after a restart)
    journal_payload_max_bytes: int = field(default=1 << 20, metadata={"env": "AI4E_JOURNAL_PAYLOAD_MAX_BYTES"})
    # image endpoints: processes that decode JPEG/PNG/npy/JSON bodies straight into the shared payload ring
    # (0 = decode on the gateway's executor threads); per endpoint: `decode_processes` in the platform YAML
    decode_processes: int = field(default=0, metadata={"env": "AI4E_DECODE_PROCESSES"})
    # ingest front-end processes sharing the public port (SO_REUSEPORT) with the serving process
    # (runtime/frontend.py); each gets `frontend_ring_slots` payload slots per GPU endpoint (0 = 4 batches)
    frontend_processes: int = field(default=0, metadata={"env": "AI4E_FRONTEND_PROCESSES"})
    frontend_ring_slots: int = field(default=0, metadata={"env": "AI4E_FRONTEND_RING_SLOTS"})
    # "native": the C++ front-end (csrc/ingest/ingestd.cpp: bodies recv()'d straight into ring slots);
    # "python": runtime/frontend.py (aiohttp). TLS listeners always use the Python front-ends.
    frontend_impl: str = field(default="native", metadata={"env": "AI4E_FRONTEND_IMPL"})
    # latency budget of an ingested request's queue wait at the native front-ends: a request whose projected wait
    # (the shard's unfinished tasks + bodies uploading + its own, over the shard's measured capacity) exceeds it is
    # answered 429 + Retry-After (0 = off: requests queue until the ring partition is full)
    max_queue_ms: float = field(default=15.0, metadata={"env": "AI4E_MAX_QUEUE_MS"})
    # control-plane shards per pool endpoint (one node scheduler + dispatch queue + ring partition each);
    # 0 = one per GPU (worker group), 1 = one scheduler for all of the endpoint's GPUs
    control_plane_shards: int = field(default=0, metadata={"env": "AI4E_CONTROL_PLANE_SHARDS"})
    # --- metrics timers (TaskQueueLogger.cs:20 / TaskProcessLogger.cs:22) ---
    queue_logger_period_s: float = field(default=30.0, metadata={"env": "AI4E_QUEUE_LOGGER_PERIOD_S"})
    process_logger_period_s: float = field(default=300.0, metadata={"env": "AI4E_PROCESS_LOGGER_PERIOD_S"})
    # --- GPU worker pool / batcher ---
    num_gpus: int = field(default=1, metadata={"env": "AI4E_NUM_GPUS"})
    max_batch: int = field(default=250, metadata={"env": "AI4E_MAX_BATCH"})  # whole waves on 256 CUs (bench.py)
    max_batch_delay_ms: float = field(default=2.0, metadata={"env": "AI4E_MAX_BATCH_DELAY_MS"})
    # graph-captured batch sizes below max_batch (low-load fast path: a batch of n runs the smallest bucket >= n)
    batch_buckets: str = field(default="8,32,128", metadata={"env": "AI4E_BATCH_BUCKETS"})
    dtype: str = field(default="bf16", metadata={"env": "AI4E_DTYPE"})
    kernel_backend: str = field(default="auto", metadata={"env": "AI4E_KERNEL_BACKEND"})  # auto|hip|torch
    use_hip_graphs: bool = field(default=True, metadata={"env": "AI4E_HIP_GRAPHS"})
    heartbeat_interval_s: float = field(default=1.0, metadata={"env": "AI4E_HEARTBEAT_S"})
    heartbeat_timeout_s: float = field(default=30.0, metadata={"env": "AI4E_HEARTBEAT_TIMEOUT_S"})
    max_batch_retries: int = field(default=3, metadata={"env": "AI4E_MAX_BATCH_RETRIES"})
    fault_injection: str = field(default="", metadata={"env": "AI4E_FAULT_INJECTION"})
    # --- gateway ---
    host: str = field(default="127.0.0.1", metadata={"env": "AI4E_HOST"})
    port: int = field(default=8080, metadata={"env": "AI4E_PORT"})
    routes_file: str = field(default="", metadata={"env": "AI4E_ROUTES"})
    sync_timeout_s: float = field(default=120.0, metadata={"env": "AI4E_SYNC_TIMEOUT_S"})
    # HTTPS listener (the Istio gateway's :443 with a mounted cert, Cluster/networking/secure_routing_base.yml):
    # PEM certificate chain + private key; both empty = plain HTTP
    tls_cert: str = field(default="", metadata={"env": "AI4E_TLS_CERT"})
    tls_key: str = field(default="", metadata={"env": "AI4E_TLS_KEY"})
    # APIM-style subscription keys (comma list) accepted on every API and task-management route, in the
    # Ocp-Apim-Subscription-Key header or the subscription-key query parameter; routes may add keys of their own
    # (`keys:` in the route table). Empty and no route keys = open access.
    subscription_keys: str = field(default="", metadata={"env": "AI4E_SUBSCRIPTION_KEYS"})
    # keys of the control routes (cache upsert/get, requests upsert/get, backend webhook, metrics/stats; the
    # reference's Function keys): besides the global keys. Once ANY key is configured (global, per route or here)
    # the control routes refuse unkeyed requests, so per-route keys alone never leave them open.
    control_keys: str = field(default="", metadata={"env": "AI4E_CONTROL_KEYS"})
    # --- autoscaler (HPA analogue, autoscaler.yaml: min/max replicas, target CURRENT_REQUESTS per replica) ---
    autoscale: bool = field(default=False, metadata={"env": "AI4E_AUTOSCALE"})
    autoscale_min_workers: int = field(default=1, metadata={"env": "AI4E_AUTOSCALE_MIN"})
    autoscale_target_per_worker: float = field(default=2.0, metadata={"env": "AI4E_AUTOSCALE_TARGET"})
    autoscale_period_s: float = field(default=5.0, metadata={"env": "AI4E_AUTOSCALE_PERIOD_S"})

    @classmethod
    def load(cls, yaml_path: Optional[str] = None, env: Optional[Dict[str, str]] = None,
             yaml_values: Optional[Dict[str, Any]] = None, **overrides: Any) -> "Config":
        env = os.environ if env is None else env
        values: Dict[str, Any] = dict(yaml_values or {})
        yaml_path = yaml_path or env.get("AI4E_CONFIG")
        if yaml_path:
            import yaml

            with open(yaml_path) as f:
                doc = yaml.safe_load(f) or {}
            values.update({k: v for k, v in doc.items() if k in {f.name for f in fields(cls)}})
        for f in fields(cls):
            name = f.metadata.get("env")
            if name and name in env:
                values[f.name] = env[name]
        values.update({k: v for k, v in overrides.items() if v is not None})
        cfg = cls()
        for f in fields(cls):
            if f.name in values:
                setattr(cfg, f.name, _coerce(f, values[f.name]))
        return cfg

    def replace(self, **kw: Any) -> "Config":
        return dataclasses.replace(self, **kw)

    def as_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


def _coerce(f: dataclasses.Field, v: Any) -> Any:
    t = f.type if isinstance(f.type, str) else getattr(f.type, "__name__", str(f.type))
    if v is None:
        return f.default
    if t == "bool":
        return _as_bool(v)
    if t == "int":
        return int(v)
    if t == "float":
        return float(v)
    return str(v)


def bucket_list(spec: Any, max_batch: int) -> List[int]:
    """Batch-size buckets for an engine: the listed sizes below ``max_batch`` plus ``max_batch`` itself.

    ``spec`` is a comma-separated string ("8,32,128") or a sequence of ints; empty = ``[max_batch]``.
    Under low load the dynamic batcher hands the engine small batches, which then run the smallest captured
    graph that fits instead of a full ``max_batch`` forward (survey §7.5 item 3).
    """
    if isinstance(spec, str):
        items = [int(x) for x in spec.replace(" ", "").split(",") if x]
    else:
        items = [int(x) for x in (spec or [])]
    return sorted({b for b in items if 0 < b < max_batch} | {int(max_batch)})


_GLOBAL: Optional[Config] = None


def get_config() -> Config:
    global _GLOBAL
    if _GLOBAL is None:
        _GLOBAL = Config.load()
    return _GLOBAL


def set_config(cfg: Config) -> None:
    global _GLOBAL
    _GLOBAL = cfg
