"""rl_games ``torch_runner.Runner`` surface used by the reference's train.py (train.py:157-178):

    runner = Runner(IsaacAlgoObserver())
    runner.algo_factory.register_builder('a2c_continuous_mirroring', lambda **kw: A2CAgentSymmetry(**kw))
    runner.load(agent_cfg); runner.reset(); runner.run({"train": True, "play": False, "sigma": None})

Seeding follows rl_games 1.6.1 ``Runner.load_config`` (torch / numpy / random from ``params.seed``).
"""

from __future__ import annotations

import copy
import random
import time

import numpy as np
import torch

from .a2c_continuous import A2CAgent, DefaultAlgoObserver
from .a2c_ppo_mirroring import A2CAgentSymmetry
from .player import PpoPlayerContinuous


class ObjectFactory:
    def __init__(self):
        self._builders: dict = {}

    def register_builder(self, name: str, builder) -> None:
        self._builders[name] = builder

    def create(self, name: str, **kwargs):
        if name not in self._builders:
            raise ValueError(f"unknown algorithm {name!r} (registered: {sorted(self._builders)})")
        return self._builders[name](**kwargs)


class Runner:
    def __init__(self, algo_observer=None):
        self.algo_factory = ObjectFactory()
        self.algo_factory.register_builder("a2c_continuous", lambda **kw: A2CAgent(**kw))
        self.algo_factory.register_builder("a2c_continuous_mirroring", lambda **kw: A2CAgentSymmetry(**kw))
        self.player_factory = ObjectFactory()
        self.player_factory.register_builder("a2c_continuous", lambda **kw: PpoPlayerContinuous(**kw))
        self.player_factory.register_builder("a2c_continuous_mirroring", lambda **kw: PpoPlayerContinuous(**kw))
        self.algo_observer = algo_observer if algo_observer is not None else DefaultAlgoObserver()
        self.agent = None

    def load_config(self, params: dict) -> None:
        self.seed = params.get("seed", None)
        if self.seed is None:
            self.seed = int(time.time())
        self.algo_name = params["algo"]["name"]
        if self.seed:
            torch.manual_seed(self.seed)
            np.random.seed(self.seed)
            random.seed(self.seed)
        params["algo_observer"] = self.algo_observer
        self.params = params

    def load(self, yaml_config: dict) -> None:
        config = copy.deepcopy(yaml_config)
        self.default_config = copy.deepcopy(config["params"])
        self.load_config(self.default_config)

    def reset(self) -> None:
        pass

    @staticmethod
    def _restore(agent, args: dict) -> None:
        ckpt = args.get("checkpoint")
        if ckpt:
            agent.restore(ckpt)

    @staticmethod
    def _override_sigma(agent, args: dict) -> None:
        sigma = args.get("sigma")
        if sigma is not None:
            with torch.no_grad():
                agent.model.a2c_network.sigma.fill_(float(sigma))

    def run_train(self, args: dict):
        self.agent = self.algo_factory.create(self.algo_name, base_name="run", params=self.params)
        self._restore(self.agent, args)
        self._override_sigma(self.agent, args)
        return self.agent.train()

    def create_player(self):
        return self.player_factory.create(self.algo_name, params=self.params)

    def run_play(self, args: dict):
        player = self.player_factory.create(self.algo_name, params=self.params)
        self._restore(player, args)
        self._override_sigma(player, args)
        return player.run()

    def run(self, args: dict):
        if args.get("train", True):
            return self.run_train(args)
        if args.get("play", False):
            return self.run_play(args)
        return self.run_train(args)
