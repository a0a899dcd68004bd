"""Agents (reference lrce/agent/__init__.py): AgentOE, AgentMC, AgentCount."""
from .agent_oe import AgentOE  # noqa: F401
from .agent_mc import AgentMC  # noqa: F401
from .agent_count import AgentCount  # noqa: F401
