from .sde_score_model import CondUNetTiny, VPSDE  # noqa: F401
