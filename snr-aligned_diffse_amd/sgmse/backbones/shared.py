from sgmse.util.registry import Registry

BackboneRegistry = Registry("Backbone")
