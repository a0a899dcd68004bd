"""Open-ended QA (reference lrce/agent/agent_oe.py): cross-entropy over the answer vocabulary with
ignore_index -100, top-1 accuracy; every other behaviour is the generic agent's."""
from .agent_base import AgentBase, get_logger


class AgentOE(AgentBase):
    def __init__(self, model, gpu_id, args, log_enabled=True, is_eval=False, rank=None):
        super().__init__(model, gpu_id, args, log_enabled, is_eval, rank)
        self.logger = get_logger(__name__, self.rank)
