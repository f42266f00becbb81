"""toycrystals_amd — MI355X-native drop-in for the hot path of sahhermans/vae-diffusion-toy-crystals.

Import the model modules as you would the reference's `toycrystals.models.*`:

    from toycrystals_amd.models.sde_score_model import CondUNetTiny, VPSDE, sample_reverse_sde_euler_maruyama
"""
__version__ = "0.1.0"
