"""MI355X-native inference engine for the Informer / Transformer channel predictors
of Bart-Hodes/ChannelEstimationTransformer."""
