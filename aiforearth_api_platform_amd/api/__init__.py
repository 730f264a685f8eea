"""Service runtime (reference layer L3): the APIService decorator API and TaskManager facade."""
from .service import APIService, RequestSnapshot
from .task_manager import DistributedApiTaskManager, HttpTaskClient, InProcTaskClient, TaskManager

__all__ = ["APIService", "RequestSnapshot", "TaskManager", "DistributedApiTaskManager", "InProcTaskClient",
           "HttpTaskClient"]
