"""GenLogger (src/ghmclip/utils/logger.py:7-36): root logger with a console
handler; with raw=False also config.log (config dump) and training.log."""
import logging
import os
from dataclasses import asdict

__all__ = ["GenLogger", "logging"]


def GenLogger(directory, config, raw=True):
    logger = logging.getLogger()
    logger.setLevel(logging.DEBUG)
    fmt = logging.Formatter('%(asctime)s - %(levelname)s - %(message)s')
    console = logging.StreamHandler()
    console.setLevel(logging.INFO)
    console.setFormatter(fmt)
    logger.addHandler(console)
    if not raw:
        os.makedirs(directory, exist_ok=True)
        cfg = logging.FileHandler(os.path.join(directory, 'config.log'), mode="a")
        cfg.setLevel(logging.DEBUG)
        cfg.setFormatter(fmt)
        train = logging.FileHandler(os.path.join(directory, 'training.log'), mode="a")
        train.setLevel(logging.DEBUG)
        train.setFormatter(fmt)
        logger.addHandler(cfg)
        logger.info(f'Training with config: {asdict(config)}')
        logger.removeHandler(cfg)
        cfg.close()
        logger.addHandler(train)
    return logger
