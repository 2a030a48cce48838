function [Pp_, Xp_, error_] = bundle_projective(Pp, Xp, x, varargin)
%BUNDLE_PROJECTIVE  Projective bundle adjustment on an AMD MI355X (vlgba drop-in).
%
%   [Pp_ Xp_ error_] = bundle_projective(Pp, Xp, x, ...)
%
%   Same signature, options and outputs as VLG's toolbox/bundle/bundle_projective.m:
%   Pp (3x4xm) projection matrices, Xp (4xn) homogeneous points (Xp(4,:) passed
%   through), x (3xnxm).  Options: 'fix_structure', 'fix_motion',
%   'visibility' V (nxm), 'verbose'.  The LM loop runs in the fused MEX gateway
%   mex_bundle_projective_lm (libvlgba on the GPU).

if nargin < 3
    help bundle_projective
    return;
end
m = size(Pp, 3);
n = size(x, 2);
opts = struct('fix_structure', 0, 'fix_motion', 0, 'verbose', 0, 'device', 0);
vis = [];
k = 1;
while k <= numel(varargin)
    name = lower(varargin{k});
    if strcmp(name, 'fix_structure'),  opts.fix_structure = 1;
    elseif strcmp(name, 'fix_motion'), opts.fix_motion = 1;
    elseif strcmp(name, 'visibility'), vis = varargin{k+1}; k = k + 1;
    elseif strcmp(name, 'verbose'),    opts.verbose = 1;
    elseif strcmp(name, 'device'),     opts.device = varargin{k+1}; k = k + 1;
    end
    k = k + 1;
end
if isempty(vis)
    vis = reshape(x(1,:,:) ~= 0 | x(2,:,:) ~= 0, n, m);
end
a = reshape(double(Pp), 12, m);             % P(:) per camera
[a, b, error_] = mex_bundle_projective_lm(a, double(Xp(1:3,:)), double(x(1:2,:,:)), ...
                                          double(vis), opts);
Pp_ = reshape(a, 3, 4, m);
Xp_ = [b; Xp(4,:)];
end
